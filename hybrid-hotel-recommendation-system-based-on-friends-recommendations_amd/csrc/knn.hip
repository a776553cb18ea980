// Cosine k-nearest-neighbour search over the item-embedding table
// (candidate generation, main.py:196-203 and /similar_items main.py:299-302,
// replacing sklearn NearestNeighbors(metric='cosine', algorithm='brute')).
//
//   dist(q, x) = clip(1 - <q/|q|, x/|x|>, 0, 2)          (fp32)
//   result: k smallest per query, ascending by (dist, row index)
//
// HBM-streaming design: the table is read exactly once per tile of QT queries.
// Each workgroup scans one contiguous row slice; every thread owns one row per
// step (16-B loads), computes QT dots against the LDS-resident normalised
// queries, and appends rows that beat the query's running k-th-best threshold
// into a per-query LDS candidate buffer.  A buffer that could overflow on the
// next step is compacted by an in-LDS bitonic sort (ties by index -> fully
// deterministic).  A second kernel merges the slices' k-lists per query.
#include "dcnr_internal.h"

#include <cfloat>
#include <climits>

namespace dcnr {
namespace {

constexpr int NT = 256;
constexpr int QT = 8;          // queries per workgroup tile
constexpr int CAP = 512;       // candidate buffer per query (>= k + NT)
constexpr int KMAX = 64;

struct Cand { float d; int i; };

__device__ __forceinline__ bool cless(float da, int ia, float db, int ib) {
  return da < db || (da == db && (unsigned)ia < (unsigned)ib);
}

// bitonic sort of CAP entries in LDS, ascending; all NT threads participate
__device__ void bitonic(float* cd, int* ci) {
  for (int k2 = 2; k2 <= CAP; k2 <<= 1) {
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < CAP / 2; t += NT) {
        int i = (t / j) * 2 * j + (t % j);
        int p = i + j;
        bool asc = (i & k2) == 0;
        float a = cd[i], b = cd[p];
        int ia = ci[i], ib = ci[p];
        bool sw = asc ? cless(b, ib, a, ia) : cless(a, ia, b, ib);
        if (sw) { cd[i] = b; cd[p] = a; ci[i] = ib; ci[p] = ia; }
      }
      __syncthreads();
    }
  }
}

// Keep the best k of buffer q: sort, pad the rest with +inf, reset count/threshold.
__device__ void compact(float* cd, int* ci, int* cnt, float* thr, int k) {
  const int n = *cnt;
  for (int t = threadIdx.x; t < CAP; t += NT)
    if (t >= n) { cd[t] = FLT_MAX; ci[t] = INT_MAX; }
  __syncthreads();
  bitonic(cd, ci);
  if (threadIdx.x == 0) {
    int kept = n < k ? n : k;
    *cnt = kept;
    *thr = kept == k ? cd[k - 1] : FLT_MAX;
  }
  __syncthreads();
}

template <int MAXV>
__global__ __launch_bounds__(NT) void scan_kernel(const float* __restrict__ tab,
                                                  const float* __restrict__ inv, int64_t N, int d,
                                                  const float* __restrict__ q, int64_t Q, int k,
                                                  int64_t rows_per_slice, Cand* out) {
  __shared__ __attribute__((aligned(16))) float qs[QT][MAXV * 4];
  __shared__ float cd[QT][CAP];
  __shared__ int ci[QT][CAP];
  __shared__ int cnt[QT];
  __shared__ float thr[QT];
  __shared__ int need;
  const int slice = blockIdx.x;
  const int64_t q0 = (int64_t)blockIdx.y * QT;
  const int nq = (int)min<int64_t>(QT, Q - q0);
  // normalised queries (sklearn normalize(): zero norm -> unchanged)
  for (int i = threadIdx.x; i < QT * MAXV * 4; i += NT) (&qs[0][0])[i] = 0.f;
  __syncthreads();
  if (threadIdx.x < 64 * QT) {
  }
  for (int qq = threadIdx.x >> 6; qq < nq; qq += NT / 64) {
    const int lane = threadIdx.x & 63;
    float s = 0.f;
    for (int i = lane; i < d; i += 64) { float v = q[(q0 + qq) * d + i]; s += v * v; }
    s = wave_sum(s);
    float in = s > 0.f ? 1.f / sqrtf(s) : 1.f;
    for (int i = lane; i < d; i += 64) qs[qq][i] = q[(q0 + qq) * d + i] * in;
  }
  if (threadIdx.x < QT) { cnt[threadIdx.x] = 0; thr[threadIdx.x] = FLT_MAX; }
  __syncthreads();

  const int64_t r0 = (int64_t)slice * rows_per_slice;
  const int64_t r1 = min(N, r0 + rows_per_slice);
  const int dv = d >> 2;
  for (int64_t base = r0; base < r1; base += NT) {
    const int64_t r = base + threadIdx.x;
    if (r < r1) {
      float4 x[MAXV];
      const float4* rp = reinterpret_cast<const float4*>(tab + r * d);
#pragma unroll
      for (int v = 0; v < MAXV; ++v) if (v < dv) x[v] = rp[v];
      const float ir = inv[r];
      for (int qq = 0; qq < nq; ++qq) {
        const float4* qp = reinterpret_cast<const float4*>(qs[qq]);
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v)
          if (v < dv) {
            float4 w = qp[v];
            s += x[v].x * w.x + x[v].y * w.y + x[v].z * w.z + x[v].w * w.w;
          }
        float dist = fminf(fmaxf(1.f - s * ir, 0.f), 2.f);
        if (dist <= thr[qq]) {
          int pos = atomicAdd(&cnt[qq], 1);
          cd[qq][pos] = dist;
          ci[qq][pos] = (int)r;
        }
      }
    }
    __syncthreads();
    for (int qq = 0; qq < nq; ++qq) {
      if (cnt[qq] > CAP - NT) compact(cd[qq], ci[qq], &cnt[qq], &thr[qq], k);
    }
  }
  (void)need;
  for (int qq = 0; qq < nq; ++qq) {
    compact(cd[qq], ci[qq], &cnt[qq], &thr[qq], k);
    Cand* o = out + ((q0 + qq) * gridDim.x + slice) * k;
    for (int t = threadIdx.x; t < k; t += NT) {
      bool ok = t < cnt[qq];
      o[t] = Cand{ok ? cd[qq][t] : FLT_MAX, ok ? ci[qq][t] : INT_MAX};
    }
  }
}

__global__ __launch_bounds__(NT) void merge_kernel(const Cand* in, int nslices, int k,
                                                   int64_t* idx, float* dist) {
  __shared__ float cd[CAP];
  __shared__ int ci[CAP];
  __shared__ int cnt;
  __shared__ float thr;
  const int64_t qq = blockIdx.x;
  const Cand* c = in + qq * (int64_t)nslices * k;
  const int total = nslices * k;
  if (threadIdx.x == 0) { cnt = 0; thr = FLT_MAX; }
  __syncthreads();
  for (int base = 0; base < total; base += NT) {
    int t = base + threadIdx.x;
    if (t < total) {
      Cand e = c[t];
      if (e.i != INT_MAX && e.d <= thr) {
        int pos = atomicAdd(&cnt, 1);
        cd[pos] = e.d;
        ci[pos] = e.i;
      }
    }
    __syncthreads();
    if (cnt > CAP - NT) compact(cd, ci, &cnt, &thr, k);
  }
  compact(cd, ci, &cnt, &thr, k);
  for (int t = threadIdx.x; t < k; t += NT) {
    bool ok = t < cnt;
    idx[qq * k + t] = ok ? (int64_t)ci[t] : -1;
    dist[qq * k + t] = ok ? cd[t] : FLT_MAX;
  }
}

__global__ void inv_norm_kernel(const float* t, int64_t N, int d, float* out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); r < N; r += nw) {
    float s = 0.f;
    for (int i = lane; i < d; i += 64) { float v = t[r * d + i]; s += v * v; }
    s = wave_sum(s);
    if (lane == 0) out[r] = s > 0.f ? 1.f / sqrtf(s) : 1.f;
  }
}

void plan(int64_t N, int64_t Q, int k, int* nslices, int64_t* rows_per_slice) {
  int64_t qtiles = cdiv(Q, QT);
  int64_t want = std::max<int64_t>(1, 2048 / qtiles);
  int64_t ns = std::min<int64_t>(want, std::max<int64_t>(1, cdiv(N, 2048)));
  *rows_per_slice = cdiv(N, ns);
  *nslices = (int)cdiv(N, *rows_per_slice);
}

}  // namespace

dcnr_status row_inv_norms(const float* t, int64_t N, int d, float* out, hipStream_t s) {
  if (N <= 0) return DCNR_OK;
  int64_t blocks = std::min<int64_t>(cdiv(N, 4), 8192);
  hipLaunchKernelGGL(inv_norm_kernel, dim3((unsigned)blocks), dim3(256), 0, s, t, N, d, out);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

size_t topk_ws(int64_t N, int64_t Q, int k) {
  int ns; int64_t rps;
  plan(N, Q, k, &ns, &rps);
  return (size_t)Q * ns * k * sizeof(Cand);
}

dcnr_status cosine_topk(const float* t, const float* inv, int64_t N, int d, const float* q,
                        int64_t Q, int k, int64_t* idx, float* dist, void* ws, size_t ws_bytes,
                        hipStream_t s) {
  if (k < 1 || k > KMAX || d < 4 || d % 4 || d > 256 || N < 1) {
    set_error("cosine_topk: unsupported k=%d d=%d N=%lld (1<=k<=64, d%%4==0, d<=256)", k, d,
              (long long)N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (Q <= 0) return DCNR_OK;
  int ns; int64_t rps;
  plan(N, Q, k, &ns, &rps);
  if (ws_bytes < topk_ws(N, Q, k)) {
    set_error("cosine_topk: workspace too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  Cand* cands = (Cand*)ws;
  dim3 grid(ns, (unsigned)cdiv(Q, QT));
  if (d <= 64)
    hipLaunchKernelGGL(scan_kernel<16>, grid, dim3(NT), 0, s, t, inv, N, d, q, Q, k, rps, cands);
  else
    hipLaunchKernelGGL(scan_kernel<64>, grid, dim3(NT), 0, s, t, inv, N, d, q, Q, k, rps, cands);
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(merge_kernel, dim3((unsigned)Q), dim3(NT), 0, s, cands, ns, k, idx, dist);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
