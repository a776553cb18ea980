// Cosine k-nearest-neighbour search over the item-embedding table
// (candidate generation, main.py:196-203 and /similar_items main.py:299-302,
// replacing sklearn NearestNeighbors(metric='cosine', algorithm='brute')).
//
//   dist(q, x) = clip(1 - <q/|q|, x/|x|>, 0, 2)          (fp32)
//   result: k smallest per query, ascending by (dist, row index)
//
// Four scans, chosen per shape in cosine_topk():
//  * scan v4 (d = 32 / 64, k <= 32; every N and Q but single queries over
//    small tables): a bf16-MFMA coarse
//    cosine over a fit-time bf16 copy of the normalised rows, with an
//    admission bound that provably keeps every true neighbour, then exact
//    fp32 distances of the admitted rows and an exact selection -- the
//    production path of configs[4] (section "scan v4" below);
//  * scan v3 (Q >= 16, d % 16 == 0, d not 32 / 64): exact fp32-MFMA scan
//    into per-slice k-lists;
//  * scan v2 (d <= 64, k <= 32): exact VALU scan with wave-register lists --
//    small Q (v4's per-query exact fallback is the same scan inside one
//    block, the same distance arithmetic);
//  * scan v1 (the rest, k <= 64): the original streaming scan below --
//    each workgroup scans one contiguous row slice; every thread owns one
//    row per step (16-B loads), computes QT dots against the LDS-resident
//    normalised queries, and appends rows that beat the query's running
//    k-th-best threshold into a per-query LDS candidate buffer, compacted
//    by an in-LDS bitonic sort (ties by index: deterministic).
// v1-v3 end in merge_kernel (the slices' k-lists per query).
#include "dcnr_internal.h"

#include <cfloat>
#include <climits>
#include <type_traits>

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

// bitonic sort of n2 (a power of two) entries in LDS, ascending by (d, i);
// all NTB threads of the block participate
template <int NTB = NT>
__device__ void bitonic(float* cd, int* ci, int n2 = CAP) {
  for (int k2 = 2; k2 <= n2; k2 <<= 1) {
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += NTB) {
        const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
        const int p = i + j;
        const bool asc = (i & k2) == 0;
        const float a = cd[i], b = cd[p];
        const int ia = ci[i], ib = ci[p];
        const bool sw = asc ? cless(b, ib, a, ia) : cless(a, ia, b, ib);
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


// The exact cosine distance's arithmetic, spelled out: x . q per float4
// chunk with the contraction fixed (fma(w, fma(z, fma(x, y-product)))), then
// 1 - s / |x| as one fma, clamped to [0, 2].  Written as plain expressions,
// the compiler picked which product to fuse -- and packed some chunks into
// v_pk_mul / v_pk_add, unfused -- differently at different call sites, so
// two scans could give one row distances an ulp apart.  Every exact-distance
// site (scan v1 / v2, the k-th bound, scan v4's epilogue, the exact
// fallbacks) sums dot4 over the chunks in order and ends with cos_dist.
__device__ __forceinline__ float dot4(const float4 x, const float4 q) {
  return fmaf(x.w, q.w, fmaf(x.z, q.z, fmaf(x.x, q.x, x.y * q.y)));
}
// dot4 of one row chunk x against two queries at once on packed fp32 math:
// qa = {q0.x, q1.x, q0.y, q1.y}, qb = {q0.z, q1.z, q0.w, q1.w} (the
// batched fallback's interleaved query layout); each lane of the result is
// dot4(x, q) bit for bit (v_pk_mul / v_pk_fma are pairs of the same ops)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 dot4_q2(const float4 x, const float4 qa, const float4 qb) {
  f32x2 p = f32x2{x.y, x.y} * f32x2{qa.z, qa.w};
  p = __builtin_elementwise_fma(f32x2{x.x, x.x}, f32x2{qa.x, qa.y}, p);
  p = __builtin_elementwise_fma(f32x2{x.z, x.z}, f32x2{qb.x, qb.y}, p);
  p = __builtin_elementwise_fma(f32x2{x.w, x.w}, f32x2{qb.z, qb.w}, p);
  return p;
}
__device__ __forceinline__ float cos_dist(float s, float ir) {
  return fminf(fmaxf(fmaf(-s, ir, 1.f), 0.f), 2.f);
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
            s += dot4(x[v], w);
          }
        float dist = cos_dist(s, ir);
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

// ---------------------------------------------------------------- scan v2
// Wave-private candidate lists (no block barriers in the scan): a block owns a
// contiguous row slice and a tile of up to K2_QT queries; each wave takes 64
// rows per step (one row per lane, in registers), computes the distance to
// every query of the tile (normalised queries broadcast from LDS), and
// appends rows that beat its running k-th best for that query with
// ballot + mbcnt (no atomics).  A full list (K2_CAP) is compacted by a
// 64-lane register bitonic sort that keeps the k best and sets the threshold.
// Rows arrive in increasing index order per wave, so the strict test
// "dist < threshold" keeps ties ordered by row index.  Output: one k-list per
// (query, block, wave), merged by merge_kernel.  Block -> (slice, query tile)
// is XCD-grouped: the blocks that share a row slice run on one XCD, whose L2
// serves the repeated reads of the slice.
constexpr int K2_NT = 256, K2_WPB = K2_NT / 64, K2_QT = 32, K2_CAP = 64, K2_KMAX = 32;
// queries from which the fp32-MFMA scan (v3) is used: measured on one box
// (tools/ab_knn.sh, 1M x 64, k = 11), the VALU scan is faster up to Q = 8
// (Q=4: 73 vs 104 us, Q=8: 97 vs 116 us), the MFMA scan from Q = 16
// (138 vs 153 us; Q=32: 189 vs 265 us)
constexpr int MFMA_MIN_Q = 16;

__device__ __forceinline__ void wave_sort64(float& d, int& i, int lane) {
#pragma unroll
  for (int k2 = 2; k2 <= 64; k2 <<= 1) {
#pragma unroll
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      const float od = __shfl_xor(d, j, 64);
      const int oi = __shfl_xor(i, j, 64);
      const bool up = (lane & k2) == 0, lower = (lane & j) == 0;
      const bool other_less = cless(od, oi, d, i);
      if ((lower == up) == other_less) { d = od; i = oi; }
    }
  }
}

// Keep the k best of one wave's list: sorted into slots [0, k).  Returns the
// new count; *kth = the k-th best distance (FLT_MAX while fewer than k).
// The list is written and read by different lanes of one wave: the wavefront
// fences order those LDS accesses for the compiler (the hardware keeps one
// wave's LDS operations in order).
__device__ __forceinline__ int wave_compact(float* cd, int* ci, int c, int k, int lane,
                                            float* kth) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  float d = lane < c ? cd[lane] : FLT_MAX;
  int i = lane < c ? ci[lane] : INT_MAX;
  wave_sort64(d, i, lane);
  if (lane < k) { cd[lane] = d; ci[lane] = i; }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const float kd = __shfl(d, k - 1, 64);
  *kth = c >= k ? kd : FLT_MAX;
  return c < k ? c : k;
}

template <int DV>
__global__ __launch_bounds__(K2_NT) void scan2_kernel(const float* __restrict__ tab,
                                                      const float* __restrict__ inv, int64_t N,
                                                      const float* __restrict__ qn, int64_t Q,
                                                      int k, int64_t rows_per_block, int nslices,
                                                      int qtiles, Cand* out,
                                                      const float* __restrict__ thr0) {
  __shared__ float cd[K2_WPB][K2_QT][K2_CAP];
  __shared__ int ci[K2_WPB][K2_QT][K2_CAP];
  __shared__ int cntl[K2_WPB][K2_QT];
  const int bid = blockIdx.x;
  const int tile = (bid / 8) % qtiles;
  const int slice = (bid % 8) + 8 * (bid / (8 * qtiles));
  if (slice >= nslices) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t q0 = (int64_t)tile * K2_QT;
  const int nq = (int)min<int64_t>(K2_QT, Q - q0);
  // the normalised queries are read with wave-uniform addresses: scalar
  // loads into SGPRs, one FMA operand each (no LDS broadcast traffic)
  const float4* qv = reinterpret_cast<const float4*>(qn + q0 * DV * 4);
  // per-query list count and threshold of this wave: lane qq holds query qq's;
  // bound0: the admission bound (kth_bound_kernel), lane qq holding query qq's
  int cntv = 0;
  float thrv = FLT_MAX;
  const float bound0 = lane < nq ? thr0[q0 + lane] : FLT_MAX;
  const int64_t r0 = (int64_t)slice * rows_per_block;
  const int64_t r1 = min(N, r0 + rows_per_block);
  for (int64_t base = r0 + 64 * w; base < r1; base += 64 * K2_WPB) {
    const int64_t r = base + lane;
    const bool ok = r < r1;
    const int64_t rc = ok ? r : r0;
    float4 x[DV];
    const float4* rp = reinterpret_cast<const float4*>(tab + rc * DV * 4);
#pragma unroll
    for (int v = 0; v < DV; ++v) x[v] = rp[v];
    const float ir = inv[rc];
    for (int qq = 0; qq < nq; ++qq) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        const float4 q = qv[qq * DV + v];
        s += dot4(x[v], q);
      }
      const float dist = cos_dist(s, ir);
      float th = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(thrv), qq));
      const float b0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bound0), qq));
      bool pass = ok && dist < th && dist <= b0;
      uint64_t m = __ballot(pass);
      if (!m) continue;
      int c = __builtin_amdgcn_readlane(cntv, qq);
      float* lcd = cd[w][qq];
      int* lci = ci[w][qq];
      while (m) {
        const int room = K2_CAP - c;
        if (room == 0) {
          c = wave_compact(lcd, lci, c, k, lane, &th);
          pass = pass && dist < th;
          m = __ballot(pass);
          continue;
        }
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (pass && rank < room) {
          lcd[c + rank] = dist;
          lci[c + rank] = (int)r;
        }
        const int n = __popcll(m);
        c += n < room ? n : room;
        pass = pass && rank >= room;
        m = __ballot(pass);
      }
      cntv = lane == qq ? c : cntv;
      thrv = lane == qq ? th : thrv;
    }
  }
  // each wave sorts its lists; then wave (qq mod 4) merges the four k-lists of
  // query qq in registers (2k <= 64 lanes per step) into the block's list
  for (int qq = 0; qq < nq; ++qq) {
    float th;
    const int c = wave_compact(cd[w][qq], ci[w][qq], __builtin_amdgcn_readlane(cntv, qq), k,
                               lane, &th);
    if (lane == 0) cntl[w][qq] = c;
  }
  __syncthreads();
  for (int qq = w; qq < nq; qq += K2_WPB) {
    float d = FLT_MAX;
    int i = INT_MAX;
    for (int ww = 0; ww < K2_WPB; ++ww) {
      const int c = cntl[ww][qq];
      const int sl = ww == 0 ? lane : lane - k;
      if (ww == 0 || lane >= k) {
        const bool has = sl >= 0 && sl < k && sl < c;
        d = has ? cd[ww][qq][sl] : FLT_MAX;
        i = has ? ci[ww][qq][sl] : INT_MAX;
      }
      if (ww > 0) wave_sort64(d, i, lane);
    }
    Cand* o = out + ((q0 + qq) * nslices + slice) * (int64_t)k;
    if (lane < k) o[lane] = Cand{d, i};
  }
}

// ---------------------------------------------------------------- scan v3
// fp32 MFMA scoring (v_mfma_f32_16x16x4_f32, exact f32 products and sums):
// per wave, 16-row tiles of the table (A operand) against K3_QT queries
// (B operand, resident in registers, 16 per column block).  The dot product
// is order-free in k, so lane (r, g) feeds k = 16 s + 4 g + j from the float4
// chunk 4 s + g of its row: every A/B fragment comes from one 16-B load, no
// shuffles.  Output lane (q, g) holds rows 4 g .. 4 g + 3 for query q.  The
// candidate lists are the per-(wave, query) LDS lists of scan v2; appends use
// ballot over the four lanes of a query; a list above K2_CAP - 16 entries is
// compacted before the next tile (at most 16 appends per tile).
constexpr int K3_QT = 32, K3_CB = K3_QT / 16;

template <int DV>
__global__ __launch_bounds__(K2_NT) void scan3_kernel(const float* __restrict__ tab,
                                                      const float* __restrict__ inv, int64_t N,
                                                      const float* __restrict__ qn, int64_t Q,
                                                      int k, int64_t rows_per_block, int nslices,
                                                      int qtiles, Cand* out,
                                                      const float* __restrict__ thr0) {
  constexpr int S4 = DV / 4;
  __shared__ float cd[K2_WPB][K3_QT][K2_CAP];
  __shared__ int ci[K2_WPB][K3_QT][K2_CAP];
  __shared__ int cntl[K2_WPB][K3_QT];
  const int bid = blockIdx.x;
  const int tile = (bid / 8) % qtiles;
  const int slice = (bid % 8) + 8 * (bid / (8 * qtiles));
  if (slice >= nslices) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t q0 = (int64_t)tile * K3_QT;
  const int nq = (int)min<int64_t>(K3_QT, Q - q0);
  float4 bq[K3_CB][S4];
#pragma unroll
  for (int cb = 0; cb < K3_CB; ++cb) {
    const int64_t qi = q0 + 16 * cb + r16;
#pragma unroll
    for (int s = 0; s < S4; ++s)
      bq[cb][s] = qi < Q ? reinterpret_cast<const float4*>(qn + qi * DV * 4)[4 * s + g]
                         : float4{0.f, 0.f, 0.f, 0.f};
  }
  float thr[K3_CB], bnd[K3_CB];
  int cnt[K3_CB];
#pragma unroll
  for (int cb = 0; cb < K3_CB; ++cb) {
    thr[cb] = FLT_MAX;
    cnt[cb] = 0;
    const int64_t qi = q0 + 16 * cb + r16;
    bnd[cb] = qi < Q ? thr0[qi] : FLT_MAX;
  }
  const uint64_t qmask = 0x0001000100010001ull << r16;
  const uint64_t below = (1ull << lane) - 1;
  const int64_t r0 = (int64_t)slice * rows_per_block;
  const int64_t r1 = min(N, r0 + rows_per_block);
  // one-tile software pipeline: the next tile's rows are in flight while this
  // tile's MFMAs and appends run
  auto load_tile = [&](int64_t b, float4 (&x)[S4], float (&v)[4]) {
    const int64_t ra = b + r16;
    const int64_t rac = ra < r1 ? ra : r0;
#pragma unroll
    for (int s = 0; s < S4; ++s) x[s] = reinterpret_cast<const float4*>(tab + rac * DV * 4)[4 * s + g];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = inv[b + 4 * g + i < r1 ? b + 4 * g + i : r0];
  };
  float4 xa[S4];
  float iv[4];
  if (r0 + 16 * w < r1) load_tile(r0 + 16 * w, xa, iv);
  for (int64_t base = r0 + 16 * w; base < r1; base += 16 * K2_WPB) {
    float4 xn[S4];
    float ivn[4];
    if (base + 16 * K2_WPB < r1) load_tile(base + 16 * K2_WPB, xn, ivn);
    const int64_t rb = base + 4 * g;
#pragma unroll
    for (int cb = 0; cb < K3_CB; ++cb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S4; ++s) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s].x, bq[cb][s].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s].y, bq[cb][s].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s].z, bq[cb][s].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s].w, bq[cb][s].w, acc, 0, 0, 0);
      }
      float* lcd = cd[w][16 * cb + r16];
      int* lci = ci[w][16 * cb + r16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dist = fminf(fmaxf(1.f - acc[i] * iv[i], 0.f), 2.f);
        const bool pass = rb + i < r1 && dist < thr[cb] && dist <= bnd[cb] && 16 * cb + r16 < nq;
        const uint64_t m = __ballot(pass);
        if (!m) continue;
        const uint64_t mq = m & qmask;
        if (pass) {
          const int slot = cnt[cb] + __popcll(mq & below);
          lcd[slot] = dist;
          lci[slot] = (int)(rb + i);
        }
        cnt[cb] += __popcll(mq);
      }
      // keep room for the next tile's (at most 16) appends per query
      uint64_t need = __ballot(lane < 16 && cnt[cb] > K2_CAP - 16);
      while (need) {
        const int q = __builtin_ctzll(need);
        need &= need - 1;
        float th;
        const int c2 = wave_compact(cd[w][16 * cb + q], ci[w][16 * cb + q],
                                    __builtin_amdgcn_readlane(cnt[cb], q), k, lane, &th);
        if (r16 == q) { cnt[cb] = c2; thr[cb] = th; }
      }
    }
#pragma unroll
    for (int s = 0; s < S4; ++s) xa[s] = xn[s];
#pragma unroll
    for (int i = 0; i < 4; ++i) iv[i] = ivn[i];
  }
#pragma unroll
  for (int cb = 0; cb < K3_CB; ++cb)
    for (int q = 0; q < 16 && 16 * cb + q < nq; ++q) {
      float th;
      const int c = wave_compact(cd[w][16 * cb + q], ci[w][16 * cb + q],
                                 __builtin_amdgcn_readlane(cnt[cb], q), k, lane, &th);
      if (lane == 0) cntl[w][16 * cb + q] = c;
    }
  __syncthreads();
  for (int qq = w; qq < nq; qq += K2_WPB) {
    float d = FLT_MAX;
    int i = INT_MAX;
    for (int ww = 0; ww < K2_WPB; ++ww) {
      const int c = cntl[ww][qq];
      const int sl = ww == 0 ? lane : lane - k;
      if (ww == 0 || lane >= k) {
        const bool has = sl >= 0 && sl < k && sl < c;
        d = has ? cd[ww][qq][sl] : FLT_MAX;
        i = has ? ci[ww][qq][sl] : INT_MAX;
      }
      if (ww > 0) wave_sort64(d, i, lane);
    }
    Cand* o = out + ((q0 + qq) * nslices + slice) * (int64_t)k;
    if (lane < k) o[lane] = Cand{d, i};
  }
}

// Per-query admission bound for the scans: the k-th smallest distance over
// the first TH_S rows of the table (+ TH_MARGIN, covering rounding differences
// between this pass and the scan kernels).  Every row of the true top-k has a
// distance <= the k-th best of any subset, so rows above the bound are never
// appended: the wave lists then see a handful of rows instead of refilling
// and re-sorting while their own thresholds converge.
constexpr int TH_S = 512;   // sample rows: the bound sits near quantile k / TH_S
constexpr float TH_MARGIN = 1e-5f;

// Block qq: normalises query qq (sklearn normalize(): zero norm -> unchanged;
// written to qn for the scan) and takes the k-th smallest sample distance by
// a 2-pass radix select over the distances' bits (exponent + 7 mantissa
// bits): the upper edge of the selected bin, an upper bound within 2^-7
// relative of the exact k-th value.
template <int DV, int NTB = 256>
__global__ __launch_bounds__(NTB) void kth_bound_kernel(const float* __restrict__ tab,
                                                        const float* __restrict__ inv, int64_t N,
                                                        const float* __restrict__ q, float* qn,
                                                        int k, float* thr0) {
  constexpr int PT = TH_S / NTB;
  constexpr int d = DV * 4;   // <= 64: one element per lane
  __shared__ unsigned hist[256];
  __shared__ unsigned sel_prefix, sel_need;
  __shared__ int sel_fail;
  __shared__ __attribute__((aligned(16))) float qs[d];
  const int64_t qq = blockIdx.x;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const float v = lane < d ? q[qq * d + lane] : 0.f;
    const float ss = wave_sum(v * v);
    const float in = ss > 0.f ? 1.f / sqrtf(ss) : 1.f;
    if (lane < d) {
      qs[lane] = v * in;
      qn[qq * d + lane] = v * in;
    }
  }
  __syncthreads();
  const float4* qv = reinterpret_cast<const float4*>(qs);
  const int S = (int)min<int64_t>(N, TH_S);
  unsigned key[PT];
#pragma unroll 4
  for (int j = 0; j < PT; ++j) {
    const int t = threadIdx.x + j * NTB;
    float dist = FLT_MAX;
    if (t < S) {
      const float4* rp = reinterpret_cast<const float4*>(tab + (int64_t)t * DV * 4);
      float4 x[DV];
#pragma unroll
      for (int v = 0; v < DV; ++v) x[v] = rp[v];
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        const float4 q = qv[v];
        s += dot4(x[v], q);
      }
      dist = cos_dist(s, inv[t]);
    }
    key[j] = __float_as_uint(dist) & 0x7fffffffu;   // >= 0: bits order like values
  }
  if (threadIdx.x == 0) { sel_prefix = 0; sel_need = (unsigned)k; sel_fail = S < k; }
  unsigned mask = 0;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int sh = 24 - 8 * pass;
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    const unsigned prefix = sel_prefix;
#pragma unroll
    for (int j = 0; j < PT; ++j)
      if ((key[j] & mask) == prefix) atomicAdd(&hist[(key[j] >> sh) & 255u], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      const unsigned need = sel_need;
      unsigned h[4], sum = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) { h[b] = hist[4 * lane + b]; sum += h[b]; }
      unsigned incl = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
      }
      unsigned cum = incl - sum;
      if (cum < need && need <= incl) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (cum + h[b] >= need) {
            sel_prefix = prefix | ((unsigned)(4 * lane + b) << sh);
            sel_need = need - cum;
            break;
          }
          cum += h[b];
        }
      }
    }
    mask |= 255u << sh;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float kth = __uint_as_float(sel_prefix | 0xffffu);
    thr0[qq] = (sel_fail || !(kth < 2.5f)) ? FLT_MAX : kth + TH_MARGIN;
  }
}

// ---------------------------------------------------------------- scan v4
// Every table and query count (d = 32 or 64): bf16-MFMA coarse scoring of
// every (row, query) pair + exact fp32 re-scoring of the rows it admits.
//
// The coarse cosine is sum_i bf16(x_i * inv_r) * bf16(q_i / |q|), fp32
// accumulation (v_mfma_f32_16x16x32_bf16: 16x the fp32-MFMA rate).  Each
// factor carries a relative rounding error <= 2^-9, so for unit vectors
// |coarse - exact| <= 2^-8 + 2^-16 + fp32 slack < V4_EPS on the distance.
// Every row of the exact top-k has exact distance <= E_k (the k-th best)
// <= T0 (the k-th best of a V4_S-row exact sample: any subset's k-th best
// bounds the table's), hence coarse distance <= T0 + V4_EPS: admitting the
// rows under that bound keeps every true neighbour, ties included.  T0 comes
// from bound5_kernel (exact distances of the sample rows, per-block k-lists,
// merged by the last-arriving block).  The admitted rows (~N k / V4_S per
// query) are appended to a per-query list with their exact fp32 distances
// (scan v2's arithmetic, computed in scan4's epilogue); rescore_kernel
// selects the k best by (distance, row) -- however many rows share the
// k-th's bin, the whole list at most.  A query whose list overflows V4_CAP
// (the count word carries V4_OVF when a block's wave list ran out of room)
// is answered by an exact scan of the whole table in rescore blocks (scan
// v2's per-wave lists and arithmetic; split over up to V4_FMAX blocks per
// query for Q <= V4_FQ): no batch-wide flag, no gated launches behind the
// chain.  Three launches per call: bound5, scan4, rescore.
constexpr float V4_EPS = 0.004f;
constexpr int V4_S = 65536;     // sample rows for the admission bound
constexpr int V4_WPS = 3;       // min waves per SIMD of scan4 for NQB > 4
constexpr int V4_CAP = 4096;     // admitted rows per query
constexpr int V4_OVF = 1 << 30;  // count-word mark: a block dropped some of this query's rows
constexpr int V4_QC = 256;       // queries per block (LDS: V4_QC x d bf16)
// table rows per block: few query blocks -> long blocks (the per-block
// prologue and epilogue amortised; measured 69 vs 78 us at Q = 32).  Many
// (NQB > 4: 16-32 KB of query fragments staged per block) -> about two blocks
// per CU, 512-2048 rows: Q = 256 over 1M rows 134 us against 146 at a fixed
// 512 (1954 blocks), 145 at 1024, 180 at 4096 (245 blocks, CUs left idle);
// profiles/lab/r04zz_knn_rpb_ab.txt.  A wave's list fill (rows x queries x
// admission rate, ~50 of 512 at 2048 rows) stays well inside V4_WL.
inline int v4_rpb(int nqb, int64_t N) {
  return nqb <= 4 ? 2048 : (int)std::min<int64_t>(2048, std::max<int64_t>(512, rup(cdiv(N, 512), 64)));
}
constexpr int64_t V4_Q1_N = 800000;   // a single query takes scan v2 below this many rows
                                      // (from Q = 2: 60-66 us for Q <= 8 against 65-98 on scan v2)

// k-th smallest of n distances (>= 0) held in LDS, by a 2-pass radix select
// over their bits (exponent + 7 mantissa bits): returns the upper edge of the
// selected bin (>= the exact k-th value, within 2^-7 relative), or
// 0xffffffff when n < k.  Every thread of the block calls it.
template <int NTB>
__device__ unsigned block_select_kth(const float* v, int n, int k) {
  __shared__ unsigned hist[256];
  __shared__ unsigned sel_prefix, sel_need;
  __shared__ int sel_fail;
  if (threadIdx.x == 0) { sel_prefix = 0; sel_need = (unsigned)k; sel_fail = n < k; }
  unsigned mask = 0;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int sh = 24 - 8 * pass;
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    const unsigned prefix = sel_prefix;
    // distances crowd into a few bins (one exponent spans a factor of 2), so
    // equal bins of a wave are counted with one atomic (up to 4 bins per
    // wave-instruction; the rest of the lanes add one each): plain per-lane
    // atomics serialised ~n times on the hottest bin
    const int lane = threadIdx.x & 63;
    for (int i0 = threadIdx.x - lane; i0 < n; i0 += NTB) {
      const int i = i0 + lane;
      const unsigned key = i < n ? __float_as_uint(v[i]) : 0u;
      const bool valid = i < n && (key & mask) == prefix;
      const unsigned bin = (key >> sh) & 255u;
      uint64_t act = __ballot(valid);
      for (int it = 0; act && it < 4; ++it) {
        const int leader = __builtin_ctzll(act);
        const unsigned lb = (unsigned)__shfl((int)bin, leader, 64);
        const uint64_t same = __ballot(valid && bin == lb) & act;
        if (lane == leader) atomicAdd(&hist[lb], (unsigned)__popcll(same));
        act &= ~same;
      }
      if ((act >> lane) & 1ull) atomicAdd(&hist[bin], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const unsigned need = sel_need;
      unsigned h[4], sum = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) { h[b] = hist[4 * lane + b]; sum += h[b]; }
      unsigned incl = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned x = __shfl_up(incl, off, 64);
        if (lane >= off) incl += x;
      }
      unsigned cum = incl - sum;
      if (cum < need && need <= incl) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (cum + h[b] >= need) {
            sel_prefix = prefix | ((unsigned)(4 * lane + b) << sh);
            sel_need = need - cum;
            break;
          }
          cum += h[b];
        }
      }
    }
    mask |= 255u << sh;
    __syncthreads();
  }
  const unsigned r = sel_fail ? 0xffffffffu : (sel_prefix | 0xffffu);
  __syncthreads();
  return r;
}

constexpr int B4_T = 1024;   // threads of the per-query v4 kernels

// one 16-row x 32-k bf16 A fragment of lane (r16, g): row r, k in
// [32 ks + 8 g, +8), scaled by the row's inverse norm
template <int KS>
__device__ __forceinline__ void v4_load_rows(const float* __restrict__ tab, int64_t r, float4 (&x)[KS][2],
                                             int g) {
  const float4* rp = reinterpret_cast<const float4*>(tab + r * (KS * 32));
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    x[ks][0] = rp[ks * 8 + 2 * g];
    x[ks][1] = rp[ks * 8 + 2 * g + 1];
  }
}

// ------------------------------------------------- scan v4 admission bound
// Replaces the round-4 sample chain (512-row bound -> sample scan -> sample
// rescore, three launches).  bound5_kernel: B5_G blocks per group of 16
// queries each score B5_C of the first V4_S table rows with scan4's coarse
// bf16 MFMA cosine and store each query's smallest coarse distance over them;
// v4_kth_bound then takes the k-th smallest M of those block minima.  k
// distinct rows (one per block) have coarse distance <= M, hence exact
// distance <= M + V4_EPS, so E_k <= T0 = M + V4_EPS: the same kind of bound
// the exact sample k-th gave (scan4 admits coarse <= T0 + V4_EPS), a rank or
// two looser when two of the sample's k best share a block.  The minima are
// merged where they are used -- in scan4's prologue for up to V4_MQ queries,
// by bound5_merge_kernel above that -- so no block waits on another (a
// last-arriving-block merge cost a device-scope release per block: 140 us
// at Q = 256, profiles/lab/r05_knn_bound_lab.txt).  Blocks of column 0 also
// write the normalised fp32 / bf16 queries (kth_bound_kernel's arithmetic)
// and zero the list counts for scan4.
constexpr int B5_C = 512;           // sample rows per block (4 waves x 8 row tiles)
constexpr int B5_G = V4_S / B5_C;   // blocks per query group (<= 128: two minima per lane)
constexpr int B5_QG = 4;            // 16-query groups per block past V4_MQ queries (rows loaded once
                                    // for them; at or under V4_MQ one group per block)
constexpr int V4_MQ = 32;           // queries up to which scan4 merges the minima itself
static_assert(B5_G <= 128, "the merge holds two block minima per lane");

// one query's ng block minima as two per lane (block g: lane g % 64, slot g / 64)
struct Mins2 { unsigned u0, u1; };
__device__ __forceinline__ Mins2 v4_load_mins(const float* mq, int ng, int lane) {
  return Mins2{lane < ng ? __float_as_uint(mq[lane]) : 0x7f7fffffu,
               lane + 64 < ng ? __float_as_uint(mq[lane + 64]) : 0x7f7fffffu};
}
// wave-wide: the admission bounds of MQ queries from their block minima:
// the k-th smallest by a bitwise search over their non-negative float bits,
// down to 10 mantissa bits, and the upper edge of that bin (>= the k-th,
// within 2^-10 relative: 5e-4 at the usual bounds against V4_EPS = 0.004).
// The MQ searches are interleaved (each step's ballot -> count -> select is
// otherwise one dependent chain).  Every lane returns the bounds.
constexpr int V4_LOWBIT = 13;
template <int MQ>
__device__ __forceinline__ void v4_kth_bounds(const Mins2 (&m)[MQ], int ng, int k, float (&out)[MQ]) {
  unsigned ans[MQ];
#pragma unroll
  for (int j = 0; j < MQ; ++j) ans[j] = 0;
  for (int b = 30; b >= V4_LOWBIT; --b) {
#pragma unroll
    for (int j = 0; j < MQ; ++j) {
      const unsigned t = ans[j] | (1u << b);
      if (__popcll(__ballot(m[j].u0 < t)) + __popcll(__ballot(m[j].u1 < t)) < k) ans[j] = t;
    }
  }
#pragma unroll
  for (int j = 0; j < MQ; ++j) {
    const float M = __uint_as_float(ans[j] | ((1u << V4_LOWBIT) - 1));
    out[j] = ng >= k && M < 2.5f ? M + V4_EPS + TH_MARGIN : FLT_MAX;
  }
}

template <int KS, bool PK, int QG>
__global__ __launch_bounds__(256) void bound5_kernel(const float* __restrict__ tab, const float* __restrict__ inv,
                                                     const bf16* __restrict__ tb, int64_t N,
                                                     const float* __restrict__ q, int64_t Q, float* qn,
                                                     bf16* qb, int* qcnt, float* mins) {
  constexpr int D = KS * 32;    // 32 or 64: one query element per lane
  constexpr int U = B5_C / 64;  // row tiles per wave
  constexpr int QB = 16 * QG;
  __shared__ __attribute__((aligned(16))) float qs[QB][D];
  __shared__ float wbest[4][QB];
  const int g = blockIdx.x;
  const int64_t q0 = (int64_t)blockIdx.y * QB;
  const int nq = (int)min<int64_t>(QB, Q - q0);
  const int ngr = (nq + 15) / 16;   // 16-query groups present
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, gl = lane >> 4;
  const int64_t S = min<int64_t>(N, V4_S);
  // the block's row tiles first (wave w: rows r0 + 16 u + r16), as scan4 loads them
  const int64_t r0 = (int64_t)g * B5_C + (B5_C / 4) * w;
  using Frag = typename std::conditional<PK, bf16x8[KS], float4[KS][2]>::type;
  Frag x[U];
  float iv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = min<int64_t>(r0 + 16 * u + r16, S - 1);
    if constexpr (PK) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) x[u][ks] = *reinterpret_cast<const bf16x8*>(tb + r * D + ks * 32 + 8 * gl);
    } else {
      v4_load_rows<KS>(tab, r, x[u], gl);
      iv[u] = inv[r];
    }
  }
  // kth_bound_kernel's normalisation, the wave's query loads all in flight first
  float qv[QB / 4];
#pragma unroll
  for (int j = 0; j < QB / 4; ++j) {
    const int qq = w + 4 * j;
    qv[j] = qq < nq && lane < D ? q[(q0 + qq) * D + lane] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < QB / 4; ++j) {
    const int qq = w + 4 * j;
    if (qq >= 16 * ngr) break;
    const float v = qv[j];
    const float ss = wave_sum(v * v);
    const float in = ss > 0.f ? 1.f / sqrtf(ss) : 1.f;
    if (lane < D) {
      qs[qq][lane] = v * in;
      if (g == 0 && qq < nq) {
        qn[(q0 + qq) * D + lane] = v * in;
        qb[(q0 + qq) * D + lane] = (bf16)(v * in);
      }
    }
    if (g == 0 && qq < nq && lane == 0) {
      qcnt[q0 + qq] = 0;
      qcnt[Q + 1 + q0 + qq] = 0;   // the fallbacks' arrival counters (rescore_kernel)
      if (q0 + qq == 0) {          // the overflow word and the batched fallback's 8 queues
        qcnt[Q] = 0;
        for (int j = 0; j < 8; ++j) qcnt[2 * Q + 2 + j] = 0;
      }
    }
  }
  __syncthreads();
  // the row tiles' A fragments (bf16, as scan4 rounds them)
  bf16x8 a[U][KS];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if constexpr (PK) {
        a[u][ks] = x[u][ks];
      } else {
        const float4 p = x[u][ks][0], v = x[u][ks][1];
        const float sc = iv[u];
        a[u][ks] = bf16x8{(bf16)(p.x * sc), (bf16)(p.y * sc), (bf16)(p.z * sc), (bf16)(p.w * sc),
                          (bf16)(v.x * sc), (bf16)(v.y * sc), (bf16)(v.z * sc), (bf16)(v.w * sc)};
      }
    }
  for (int gr = 0; gr < ngr; ++gr) {
    // B fragment of lane (c = r16, gl): query 16 gr + c's k-chunk [32 ks + 8 gl, +8)
    bf16x8 bq[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const float4 lo = *reinterpret_cast<const float4*>(&qs[16 * gr + r16][ks * 32 + 8 * gl]);
      const float4 hi = *reinterpret_cast<const float4*>(&qs[16 * gr + r16][ks * 32 + 8 * gl + 4]);
      bq[ks] = bf16x8{(bf16)lo.x, (bf16)lo.y, (bf16)lo.z, (bf16)lo.w, (bf16)hi.x, (bf16)hi.y, (bf16)hi.z, (bf16)hi.w};
    }
    // best coarse cosine of each query over the block's rows
    float best = -FLT_MAX;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][ks], bq[ks], acc, 0, 0, 0);
      // lane (c, gl): rows r0 + 16 u + 4 gl + i of query c
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (r0 + 16 * u + 4 * gl + i < S) best = fmaxf(best, acc[i]);
    }
    best = fmaxf(best, __shfl_xor(best, 16, 64));
    best = fmaxf(best, __shfl_xor(best, 32, 64));
    if (lane < 16) wbest[w][16 * gr + lane] = best;
  }
  __syncthreads();
  if (threadIdx.x < nq) {
    const int c = threadIdx.x;
    const float bc = fmaxf(fmaxf(wbest[0][c], wbest[1][c]), fmaxf(wbest[2][c], wbest[3][c]));
    // (clamped at 0, which only raises a minimum and so keeps the bound valid)
    mins[(q0 + c) * B5_G + g] = fmaxf(1.f - bc, 0.f);
  }
}

// more than V4_MQ queries: one wave per query merges its minima into thr0
__global__ __launch_bounds__(256) void bound5_merge_kernel(const float* __restrict__ mins, int ng, int64_t Q,
                                                           int k, float* thr0) {
  const int64_t qq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qq >= Q) return;
  const Mins2 m[1] = {v4_load_mins(mins + qq * B5_G, ng, threadIdx.x & 63)};
  float t[1];
  v4_kth_bounds<1>(m, ng, k, t);
  if ((threadIdx.x & 63) == 0) thr0[qq] = t[0];
}

// Admissions go to a wave-private LDS list whose fill count is wave-uniform
// (ballots + mbcnt, no atomic at all inside the loop: a returning global
// atomic there put its contended round trip in every tile, a returning LDS
// atomic ~100 cycles per admitting check).  At the end the block counts its
// entries per query, reserves each query's range with one global atomic per
// (block, query), and scatters.
constexpr int V4_LIST = 2048;    // admitted (query, row) pairs per block
constexpr int V4_WL = V4_LIST / 4;   // ... per wave
constexpr int V4_PF = 4;        // packed row tiles in flight per wave

// (NQB > 4: at least 3 waves per SIMD -- left alone the compiler unrolled
// its way to 284 registers and one wave per SIMD, 1.7x slower)
template <int KS, int NQB, bool PK>
__global__ __launch_bounds__(256, NQB > 4 ? V4_WPS : 1) void scan4_kernel(const float* __restrict__ tab,
                                                    const float* __restrict__ inv,
                                                    const bf16* __restrict__ tb, int64_t N, int rpb,
                                                    const bf16* __restrict__ qb,
                                                    const float* __restrict__ thr0,
                                                    const float* __restrict__ qn, int64_t Q, int* qcnt,
                                                    int* rows, float* dists,
                                                    const float* __restrict__ bmins, int ng, int k) {
  constexpr int D = KS * 32;
  // up to 4 query blocks the B fragments live in registers; beyond that
  // (64+ KS x 4 VGPRs) in LDS, stored in fragment order -- entry (b, ks,
  // lane) is lane's 16 B, so a wave's ds_read_b128 is one contiguous 1 KB
  // with no bank conflicts.  (Left to itself the compiler re-loaded the
  // register copy from global memory every tile.)
  constexpr bool BL = NQB > 4;
  __shared__ int lq[V4_LIST];     // admitted (query, row) pairs of the block
  __shared__ int lr[V4_LIST];
  __shared__ int qn_[NQB * 16];   // per-query counts, then this block's bases
  __shared__ float thl[NQB * 16]; // (bmins) the block's admission bounds
  __shared__ int wcnt[4];
  __shared__ bf16x8 bqs[BL ? NQB * KS * 64 : 1];
  const int64_t qc0 = (int64_t)blockIdx.y * (NQB * 16);
  const int nq = (int)min<int64_t>(NQB * 16, Q - qc0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(N, r0 + rpb);
  // A fragments of the next PF row tiles in flight per wave (a register
  // ring, static indices): fp32 rows scaled and rounded here, or (PK) the
  // fit-time bf16 copy loaded as is.  The first PF loads go out before the
  // query fragments are staged.
  constexpr int PF = PK && NQB <= 4 ? V4_PF : 2;
  using Frag = typename std::conditional<PK, bf16x8[KS], float4[KS][2]>::type;
  Frag x[PF];
  float iv[PF];
  auto load = [&](int64_t bse, Frag& xx, float& ivv) {
    if (bse < r1) {
      const int64_t r = bse + r16 < r1 ? bse + r16 : r0;
      if constexpr (PK) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) xx[ks] = *reinterpret_cast<const bf16x8*>(tb + r * D + ks * 32 + 8 * g);
      } else {
        v4_load_rows<KS>(tab, r, xx, g);
        ivv = inv[r];
      }
    }
  };
  // (bound5 minima to merge: loaded before everything else, so the merge
  // waits for them alone and runs under the row tiles' loads)
  constexpr int MWMAX = NQB * 16 <= V4_MQ ? NQB * 16 / 4 : 1;
  Mins2 mm[MWMAX];
  if constexpr (NQB * 16 <= V4_MQ) if (bmins) {
#pragma unroll
    for (int j = 0; j < MWMAX; ++j) mm[j] = v4_load_mins(bmins + (qc0 + min(w + 4 * j, nq - 1)) * B5_G, ng, lane);
  }
  const int64_t first = r0 + 16 * w;
#pragma unroll
  for (int u = 0; u < PF; ++u) load(first + 64 * u, x[u], iv[u]);
  int wc = 0;   // this wave's list fill (wave-uniform)
  // lane (c = r16, g) of B fragment (b, ks): query 16 b + c's k-chunk
  // [32 ks + 8 g, +8)
  bf16x8 bq[BL ? 1 : NQB][KS];
  float th[NQB];
  // (clamped indices + selects: all of these loads are in flight at once --
  // as guarded loads the compiler issued them one round trip at a time,
  // 16 serial misses in the prologue of every NQB = 16 block)
#pragma unroll
  for (int b = 0; b < NQB; ++b) {
    const int qi = 16 * b + r16;
    const int64_t qs = qc0 + min(qi, nq - 1);
    if constexpr (!BL) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(qb + qs * D + ks * 32 + 8 * g);
        bq[b][ks] = qi < nq ? v : bf16x8{};
      }
    }
    if (!bmins) {
      const float t = thr0[qs];   // (bound5_merge_kernel's)
      // a row passes iff its coarse cosine is >= 1 - bound; the 1e-6 below
      // covers the rounding of 1 - bound (query slots past nq: 2, never)
      th[b] = qi < nq ? (1.f - (t + V4_EPS)) - 1e-6f : 2.f;
    }
  }
  // few queries (V4_MQ: NQB = 2): merge their bound5 minima here, a wave per query
  if constexpr (NQB * 16 <= V4_MQ) if (bmins) {
    auto merge = [&](auto mw_c) {
      constexpr int MW = decltype(mw_c)::value;   // queries per wave
      Mins2 m2[MW];
#pragma unroll
      for (int j = 0; j < MW; ++j) m2[j] = mm[j];
      float tj[MW];
      v4_kth_bounds<MW>(m2, ng, k, tj);
#pragma unroll
      for (int j = 0; j < MW; ++j) {
        const int qq = w + 4 * j;
        if (qq < nq && lane == 0) thl[qq] = tj[j];
      }
    };
    if (nq <= 4) merge(std::integral_constant<int, 1>{});
    else if (nq <= 16) merge(std::integral_constant<int, 4>{});
    else merge(std::integral_constant<int, NQB * 16 / 4>{});
  }
  if constexpr (BL) {
    constexpr int PER = NQB * KS * 64 / 256;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = threadIdx.x + 256 * j;
      const int l = e & 63, ks = (e >> 6) % KS, b = (e >> 6) / KS;
      const int qi = 16 * b + (l & 15);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(qb + (qc0 + min(qi, nq - 1)) * D + ks * 32 + 8 * (l >> 4));
      bqs[e] = qi < nq ? v : bf16x8{};
    }
  }
  for (int i = threadIdx.x; i < NQB * 16; i += 256) qn_[i] = 0;
  __syncthreads();
  if constexpr (NQB * 16 <= V4_MQ) if (bmins) {
#pragma unroll
    for (int b = 0; b < NQB; ++b) {
      const int qi = 16 * b + r16;
      th[b] = qi < nq ? (1.f - (thl[qi] + V4_EPS)) - 1e-6f : 2.f;
    }
  }
  for (int64_t b0 = first; b0 < r1; b0 += 64 * PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int64_t base = b0 + 64 * u;
      if (base >= r1) break;
      bf16x8 a[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if constexpr (PK) {
          a[ks] = x[u][ks];
        } else {
          const float4 p = x[u][ks][0], v = x[u][ks][1];
          const float s = iv[u];
          a[ks] = bf16x8{(bf16)(p.x * s), (bf16)(p.y * s), (bf16)(p.z * s), (bf16)(p.w * s),
                         (bf16)(v.x * s), (bf16)(v.y * s), (bf16)(v.z * s), (bf16)(v.w * s)};
        }
      }
      load(base + 64 * PF, x[u], iv[u]);
      // every query block's MFMAs first, back to back (interleaving each
      // block's admission checks serialised LDS read -> MFMA -> result ->
      // ballot per block: 146 us for 256 queries), then one ballot per block
      // on the best of its 4 rows -- usually empty -- before the per-row
      // ones.  The accumulators start at bound - 1, so a check is a sign
      // test: with |coarse - exact| <= 2^-8 + 2^-16 + fp32 accumulation error
      // (< 1e-5 here) against V4_EPS = 0.004 the admitted set still contains
      // every row whose exact distance is <= the bound.
      // (LDS fragments: block b + 1's read is issued before block b's MFMAs)
      f32x4 acc[NQB];
      bf16x8 nb[KS];
      if constexpr (BL) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) nb[ks] = bqs[ks * 64 + lane];
      }
#pragma unroll
      for (int b = 0; b < NQB; ++b) {
        bf16x8 cb[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) cb[ks] = BL ? nb[ks] : bq[BL ? 0 : b][ks];
        if constexpr (BL) {
          if (b + 1 < NQB) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) nb[ks] = bqs[((b + 1) * KS + ks) * 64 + lane];
          }
        }
        acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], cb[ks], acc[b], 0, 0, 0);
      }
      const bool full = base + 16 <= r1;   // (wave-uniform) no row of the tile past r1
      const int rb = (int)base + 4 * g;
#pragma unroll
      for (int b = 0; b < NQB; ++b) {
        // lane (c = r16, g): rows rb + i, query 16 b + c
        const float mx = fmaxf(fmaxf(acc[b][0], acc[b][1]), fmaxf(acc[b][2], acc[b][3]));
        if (!__ballot(mx >= th[b])) continue;
        // one block adds at most 256 entries: room is checked once here (a
        // full list reads as overflowed, and the batch takes the exact path)
        if (wc > V4_WL - 256) { wc = V4_WL + 1; continue; }
        int* lqw = lq + w * V4_WL;
        int* lrw = lr + w * V4_WL;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool pass = acc[b][i] >= th[b] && (full || rb + i < r1);
          const uint64_t m = __ballot(pass);
          if (pass) {
            const int p = wc + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            lqw[p] = 16 * b + r16;
            lrw[p] = rb + i;
          }
          wc += __popcll(m);
        }
      }
    }
  }
  if (lane == 0) wcnt[w] = wc;
  __syncthreads();
  const int c0 = wcnt[0], c1 = wcnt[1], c2 = wcnt[2], c3 = wcnt[3];
  if (max(max(c0, c1), max(c2, c3)) > V4_WL) {   // a wave's list overflowed: every query
    for (int q = threadIdx.x; q < nq; q += 256)     // of the block takes the exact path
      atomicOr(&qcnt[qc0 + q], V4_OVF);
    if (threadIdx.x == 0) qcnt[Q] = 1;              // the call's overflow word
    return;
  }
  // entry j of the block (waves' lists back to back) -> its LDS slot
  const int s1 = c0, s2 = c0 + c1, s3 = c0 + c1 + c2, n = s3 + c3;
  auto slot = [&](int j) {
    return j < s1 ? j : j < s2 ? V4_WL + j - s1 : j < s3 ? 2 * V4_WL + j - s2 : 3 * V4_WL + j - s3;
  };
  for (int e = threadIdx.x; e < n; e += 256) atomicAdd(&qn_[lq[slot(e)]], 1);
  __syncthreads();
  for (int q = threadIdx.x; q < nq; q += 256) {
    const int c = qn_[q];
    qn_[q] = c ? atomicAdd(&qcnt[qc0 + q], c) : 0;   // this block's range of query q's list
    if (c && qn_[q] + c > V4_CAP) qcnt[Q] = 1;       // the list overflowed: the call's overflow word
  }
  __syncthreads();
  // exact fp32 distance of every admitted pair, here rather than in the
  // per-query rescore: the row gathers then overlap the other blocks'
  // streaming instead of forming a one-block-per-query latency chain.  One
  // lane per pair, the float4 chunks summed in order: scan v2's arithmetic,
  // expression for expression, so v2 and v4 give a row the same distance
  // bit for bit (a row-sharded index, whose small shards may take v2, then
  // returns the single index's answer).
  constexpr int DV = KS * 8;
  const float4* tab4 = reinterpret_cast<const float4*>(tab);
  const float4* qn4 = reinterpret_cast<const float4*>(qn);
  for (int e = threadIdx.x; e < n; e += 256) {
    const int sl = slot(e);
    const int qe = lq[sl], re = lr[sl];
    const float4* rp = tab4 + (int64_t)re * DV;
    const float4* qp = qn4 + (qc0 + qe) * DV;
    float4 x[DV];
#pragma unroll
    for (int v = 0; v < DV; ++v) x[v] = rp[v];
    const float ir = inv[re];
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < DV; ++v) {
      const float4 q = qp[v];
      s += dot4(x[v], q);
    }
    const float dist = cos_dist(s, ir);
    const int pos = atomicAdd(&qn_[qe], 1);
    if (pos < V4_CAP) {   // (past it the query's count exceeds V4_CAP: exact path)
      const int64_t o = (qc0 + qe) * V4_CAP + pos;
      rows[o] = re;
      dists[o] = dist;
    }
  }
}


// Exact top-k of one query over the whole table inside one B4_T-thread block:
// scan v2's per-wave lists (rows in increasing order per wave, admitted while
// strictly under the wave's k-th best, compacted by a register bitonic sort)
// and its distance arithmetic expression for expression, then wave 0 merges
// the waves' sorted k-lists.  The same (distance, row) order as every other
// scan, so a query that lands here returns what scan v2 returns.  Needs
// k <= 32 (two k-lists per 64-lane merge step) and 16 * 64 * 8 B of LDS.
// scan v2's exact distance of one row (x, its inverse norm ir) to one
// normalised query (wave-uniform qv): the one expression every exact path
// uses, so they agree bit for bit
template <int DV>
__device__ __forceinline__ float exact_dist(const float4 (&x)[DV], const float4* qv, float ir) {
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < DV; ++v) {
    const float4 q = qv[v];
    s += dot4(x[v], q);
  }
  return cos_dist(s, ir);
}

// admit (dd, r) into one wave's k-list (64 LDS slots, compacted when full)
// while strictly under its k-th best: scan v2's per-wave list protocol
__device__ __forceinline__ void wave_admit(float* lcd, int* lci, int& c, float& th, int k, int lane,
                                           bool ok, float dd, int64_t r) {
  bool pass = ok && dd < th;
  uint64_t m = __ballot(pass);
  while (m) {
    const int room = 64 - c;
    if (room == 0) {
      c = wave_compact(lcd, lci, c, k, lane, &th);
      pass = pass && dd < th;
      m = __ballot(pass);
      continue;
    }
    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    if (pass && rank < room) {
      lcd[c + rank] = dd;
      lci[c + rank] = (int)r;
    }
    const int n = __popcll(m);
    c += n < room ? n : room;
    pass = pass && rank >= room;
    m = __ballot(pass);
  }
}

// merge NW sorted wave k-lists (wave ww's at cd[ww * 64], ci[ww * 64], counts
// cnt[ww]) in one wave: the k best by (distance, row) in lanes [0, k)
template <int NW>
__device__ __forceinline__ void wave_merge_lists(const float* cd, const int* ci, const int* cnt, int k,
                                                 int lane, float& d, int& i) {
  d = FLT_MAX;
  i = INT_MAX;
  for (int ww = 0; ww < NW; ++ww) {
    const int cw = cnt[ww];
    const int sl = ww == 0 ? lane : lane - k;
    if (ww == 0 || lane >= k) {
      const bool has = sl >= 0 && sl < k && sl < cw;
      d = has ? cd[ww * 64 + sl] : FLT_MAX;
      i = has ? ci[ww * 64 + sl] : INT_MAX;
    }
    if (ww > 0) wave_sort64(d, i, lane);
  }
}

template <int DV>
__device__ void exact_query_topk(const float* __restrict__ tab, const float* __restrict__ inv, int64_t lo,
                                 int64_t N, const float* __restrict__ qrow, int k, float* lds, int64_t* idx,
                                 float* dist) {
  constexpr int NW = B4_T / 64;
  __shared__ int cntl[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* lcd = lds + w * 64;
  int* lci = reinterpret_cast<int*>(lds + NW * 64) + w * 64;
  // wave-uniform addresses: the query comes in through scalar loads
  const float4* qv = reinterpret_cast<const float4*>(qrow);
  int c = 0;
  float th = FLT_MAX;
  for (int64_t base = lo + 64 * w; base < N; base += 64 * NW) {   // rows [lo, N)
    const int64_t r = base + lane;
    const bool ok = r < N;
    const int64_t rc = ok ? r : 0;
    float4 x[DV];
    const float4* rp = reinterpret_cast<const float4*>(tab + rc * DV * 4);
#pragma unroll
    for (int v = 0; v < DV; ++v) x[v] = rp[v];
    const float dd = exact_dist<DV>(x, qv, inv[rc]);
    wave_admit(lcd, lci, c, th, k, lane, ok, dd, r);
  }
  c = wave_compact(lcd, lci, c, k, lane, &th);
  if (lane == 0) cntl[w] = c;
  __syncthreads();
  if (w == 0) {
    float d;
    int i;
    wave_merge_lists<NW>(lds, reinterpret_cast<const int*>(lds + NW * 64), cntl, k, lane, d, i);
    if (lane < k) {
      idx[lane] = (int64_t)i;
      dist[lane] = d;
    }
  }
}

// The batched exact fallback (Q > V4_FQ): work item (group h of V4_BQ
// queries, row chunk f) scans rows [lo, hi) once for every overflowed query
// of the group -- each wave holds a row in registers and scores it against
// each of them (exact_dist: the single-query scan's bits), one k-list per
// (query, wave) -- then the block's waves merge query qi's wave lists into
// the item's k-list for that query.  The table is read once per group
// of V4_BQ queries instead of once per query.
constexpr int V4_BQ = 8;      // queries per batch work item
template <int DV, int BT>
__device__ void exact_batch_item(const float* __restrict__ tab, const float* __restrict__ inv, int64_t lo,
                                 int64_t hi, const float* __restrict__ qg, unsigned act, int k,
                                 float* bcd, int* bci, int* bcnt, float* bq, float* pd, int64_t* pi,
                                 int64_t lstride) {
  constexpr int NW = BT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the group's queries, interleaved by pairs: chunk v of pair pr at
  // bq[(pr DV + v) 8 ..] = q0.x q1.x q0.y q1.y q0.z q1.z q0.w q1.w
  for (int e = threadIdx.x; e < V4_BQ * DV * 4; e += BT) {
    const int pr = e / (DV * 8), r = e % (DV * 8), v = r / 8, c = (r % 8) / 2, o = r % 2;
    bq[e] = qg[(2 * pr + o) * DV * 4 + v * 4 + c];
  }
  __syncthreads();
  // query qi's list count and k-th best live in lane qi (two VGPRs, not
  // 2 x V4_BQ scalars: the kernel's SGPRs are already full)
  int cv = 0;
  float thv = FLT_MAX;
  for (int64_t base = lo + 64 * w; base < hi; base += 64 * NW) {
    const int64_t r = base + lane;
    const bool ok = r < hi;
    const int64_t rc = ok ? r : lo;
    const float4* rp = reinterpret_cast<const float4*>(tab + rc * DV * 4);
    const float ir = ((const __attribute__((address_space(1))) float*)inv)[rc];
    // the V4_BQ distances, float4 chunk by chunk (each query's sum in
    // exact_dist's order: dot4 per chunk, in order; two queries per packed
    // op); the queries come from the LDS copy (uniform-address reads into
    // VGPRs: as scalar loads the compiler hoists them into 4 DV V4_BQ SGPRs
    // and spills)
    float sq[V4_BQ];
#pragma unroll
    for (int qi = 0; qi < V4_BQ; ++qi) sq[qi] = 0.f;
    // the whole row first: its DV loads in flight together (global address
    // space: a flat load would also count against the LDS reads' waits)
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) f32x4v gf32x4;
    float4 x[DV];
#pragma unroll
    for (int v = 0; v < DV; ++v) {
      const f32x4v t = ((gf32x4*)rp)[v];
      x[v] = make_float4(t.x, t.y, t.z, t.w);
    }
    const float4* bq4 = reinterpret_cast<const float4*>(bq);
#pragma unroll
    for (int v = 0; v < DV; ++v) {
      const float4 xv = x[v];
#pragma unroll
      for (int pr = 0; pr < V4_BQ / 2; ++pr) {
        const f32x2 p = dot4_q2(xv, bq4[(pr * DV + v) * 2], bq4[(pr * DV + v) * 2 + 1]);
        sq[2 * pr] += p.x;
        sq[2 * pr + 1] += p.y;
      }
    }
#pragma unroll
    for (int qi = 0; qi < V4_BQ; ++qi) sq[qi] = cos_dist(sq[qi], ir);
#pragma unroll 1
    for (int qi = 0; qi < V4_BQ; ++qi) {
      if (!((act >> qi) & 1u)) continue;   // (uniform)
      float dd = sq[0];
#pragma unroll
      for (int j = 1; j < V4_BQ; ++j) dd = qi == j ? sq[j] : dd;
      int c = __builtin_amdgcn_readlane(cv, qi);
      float th = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(thv), qi));
      wave_admit(bcd + (qi * NW + w) * 64, bci + (qi * NW + w) * 64, c, th, k, lane, ok, dd, r);
      cv = lane == qi ? c : cv;
      thv = lane == qi ? th : thv;
    }
  }
#pragma unroll
  for (int qi = 0; qi < V4_BQ; ++qi) {
    if (!((act >> qi) & 1u)) continue;
    float th = 0.f;
    const int cc = wave_compact(bcd + (qi * NW + w) * 64, bci + (qi * NW + w) * 64,
                                __builtin_amdgcn_readlane(cv, qi), k, lane, &th);
    if (lane == 0) bcnt[qi * NW + w] = cc;
  }
  __syncthreads();
  for (int qi = w; qi < V4_BQ; qi += NW) {
    if (!((act >> qi) & 1u)) continue;
    float d;
    int i;
    wave_merge_lists<NW>(bcd + qi * NW * 64, bci + qi * NW * 64, bcnt + qi * NW, k, lane, d, i);
    if (lane < k) {
      pd[qi * lstride + lane] = d;
      pi[qi * lstride + lane] = (int64_t)i;
    }
  }
}

// The batched fallback's work pool (Q > V4_FQ).  scan4 raises the call's
// overflow word (qcnt[Q]) when any query's list overflows; then every
// rescore block, its own query done, pulls work items from a queue word
// (qcnt[2Q + 1]) until they run out.  Item it = (row chunk it / H, group
// it % H): consecutive items share a chunk, so blocks pulling together read
// the same rows.  An item scans its chunk for the group's overflowed queries
// (exact_batch_item); the last of a group's FB items merges each overflowed
// query's FB k-lists.  Not inlined, so the per-query path keeps its
// registers (inlined, the kernel spilled SGPRs).  A call with nothing
// overflowed never enters it: no extra blocks, one extra word read per block.
template <int DV>
__device__ __attribute__((noinline)) void batch_fallback_pool(
    const int* qcnt, int* heads, int k, int64_t* idx, float* dist, const float* __restrict__ tab,
    const float* __restrict__ inv, int64_t N, const float* __restrict__ qn, int64_t Q, int FB, float* pd,
    int64_t* pi, int* pcnt, float* bcd, int* bci, int* bcnt, float* bq, int* slot) {
  constexpr int NW = B4_T / 64;
  const int64_t H = (Q + V4_BQ - 1) / V4_BQ;
  // queue g = blockIdx % 8 holds the chunks f = g (mod 8): blocks sharing an
  // XCD share its queue, so a chunk (<= ~2 MB) is read from HBM once and its
  // groups' items hit that XCD's L2 (speed only: every queue has blocks
  // -- Q > 16 -- and every block joins when the overflow word is up)
  const int g = (int)(blockIdx.x % 8);
  const int64_t items = H * (FB / 8);
  for (;;) {
    __syncthreads();   // (the LDS lists and the slot word are reused)
    if (threadIdx.x == 0) *slot = atomicAdd(heads + g, 1);
    __syncthreads();
    const int64_t it = *slot;
    if (it >= items) return;
    const int fb = g + 8 * (int)(it / H);
    const int64_t h = it % H, q0 = h * V4_BQ;
    unsigned act = 0;
    for (int qi = 0; qi < V4_BQ && q0 + qi < Q; ++qi) {
      const int n = qcnt[q0 + qi];
      if (n > V4_CAP || n < k) act |= 1u << qi;
    }
    if (!act) continue;
    const int64_t lo = N * fb / FB, hi = N * (fb + 1) / FB;
    exact_batch_item<DV, B4_T>(tab, inv, lo, hi, qn + q0 * DV * 4, act, k, bcd, bci, bcnt, bq,
                               pd + (q0 * FB + fb) * k, pi + (q0 * FB + fb) * k, (int64_t)FB * k);
    if (last_arriver(pcnt + h, FB, slot)) {
      // the group's last item: its waves merge the overflowed queries' FB k-lists
      const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
      for (int qi = w; qi < V4_BQ; qi += NW) {
        if (!((act >> qi) & 1u)) continue;
        const int64_t qq = q0 + qi;
        float d = FLT_MAX;
        int i = INT_MAX;
        for (int ff = 0; ff < FB; ++ff) {
          const int sl = ff == 0 ? lane : lane - k;
          if (ff == 0 || lane >= k) {
            const bool has = sl >= 0 && sl < k;
            const float dv = has ? pd[(qq * FB + ff) * k + sl] : FLT_MAX;
            const int64_t iv = has ? pi[(qq * FB + ff) * k + sl] : (int64_t)INT_MAX;
            d = dv;
            i = dv == FLT_MAX ? INT_MAX : (int)iv;
          }
          if (ff > 0) wave_sort64(d, i, lane);
        }
        if (lane < k) {
          idx[qq * k + lane] = (int64_t)i;
          dist[qq * k + lane] = d;
        }
      }
    }
  }
}

// One block per query: the exact distances of its admitted rows (computed
// by scan4's epilogue), the k-th smallest by block_select_kth, then a bitonic
// sort of the rows at or under the selected bin by (distance, row).  A query
// whose list overflowed takes exact_query_topk (DV = d / 4) -- with few
// queries (F > 1: blocks q + Q f, f = 1 .. F-1, that return at once unless
// q's list overflowed) split over F blocks, each scanning 1/F of the table
// into a k-list, the last-arriving one merging them: the all-overflow call
// (a table with thousands of duplicates per query) no longer puts the whole
// table through one CU (the merge keeps the (distance,
// row) order, so the answer is the single block's bit for bit).
constexpr int V4_FMAX = 64;        // fallback blocks per query
constexpr int V4_FQ = 16;          // queries up to which the fallback is split
inline int v4_fallback_split(int64_t Q) {
  return Q <= V4_FQ ? (int)std::min<int64_t>(V4_FMAX, 256 / Q) : 1;
}
// Q > V4_FQ: row chunks of the batched fallback (about V4_BI work items,
// 8..128 chunks, a multiple of 8); 0: none.  Few large items: all-overflow
// Q = 256 over 1M x 64 took 1.27 / 1.34 / 1.57 / 1.93 / 2.67 ms at 256 / 512 /
// 1024 / 2048 / 4096 items (profiles/lab/r06_knn_batch_lab.txt).  The
// k-lists: Q x chunks x 32 x 12 B, ~12 MB at most.
constexpr int V4_BI = 256;
inline int v4_batch_chunks(int64_t Q) {
  if (Q <= V4_FQ) return 0;
  const int64_t H = (Q + V4_BQ - 1) / V4_BQ;
  return (int)std::max<int64_t>(8, std::min<int64_t>(128, (V4_BI / H) / 8 * 8));
}
// k-lists per query of either fallback form
inline int v4_lists(int64_t Q) {
  const int F = v4_fallback_split(Q);
  return F > 1 ? F : v4_batch_chunks(Q);
}
template <int DV>
__global__ __launch_bounds__(B4_T) void rescore_kernel(const float* __restrict__ dists, const int* qcnt,
                                                       const int* rows, int k, int64_t* idx,
                                                       float* dist, const float* __restrict__ tab,
                                                       const float* __restrict__ inv, int64_t N,
                                                       const float* __restrict__ qn, int64_t Q, int F,
                                                       int FB, float* pd, int64_t* pi, int* pcnt) {
  // one LDS image: dl / cd / ci of the per-query path, or the batched
  // fallback's (query, wave) lists (FB > 0: blocks from Q on, which answer
  // the overflowed queries)
  constexpr int NW = B4_T / 64;
  constexpr int BL = V4_BQ * NW * 64;
  constexpr int SMW = 3 * V4_CAP > 2 * BL ? 3 * V4_CAP : 2 * BL;
  __shared__ float smem[SMW];
  __shared__ int bcnt[V4_BQ * NW];
  __shared__ float bq[V4_BQ * 64];   // the batched fallback's queries (d <= 64)
  float* dl = smem;
  float* cd = smem + V4_CAP;   // the rows at or under the k-th's bin: all of the list at most
  int* ci = reinterpret_cast<int*>(smem + 2 * V4_CAP);
  __shared__ int cnt;
  __shared__ int last;
  static_assert(V4_CAP >= 2 * B4_T, "exact fallback lists live in dl");
  // FB > 0: the batched fallback's pool, entered after this block's own
  // query when scan4 raised the overflow word (or this query overflowed)
  const bool pool = FB > 0 && qcnt[Q] != 0;
  auto join_pool = [&]() {
    batch_fallback_pool<DV>(qcnt, const_cast<int*>(qcnt) + 2 * Q + 2, k, idx, dist, tab, inv, N, qn, Q, FB, pd,
                            pi, pcnt, smem, reinterpret_cast<int*>(smem + BL), bcnt, bq, &last);
  };
  const int64_t qq = blockIdx.x % Q;
  const int f = (int)(blockIdx.x / Q);
  auto fail = [&]() {
    __syncthreads();   // (dl is reused)
    exact_query_topk<DV>(tab, inv, 0, N, qn + qq * DV * 4, k, dl, idx + qq * k, dist + qq * k);
  };
  // the split fallback: rows [N f / F, N (f+1) / F) -> k-list f of the query,
  // then the last of its F blocks merges the F lists (wave 0)
  auto split = [&]() {
    __syncthreads();
    const int64_t lo = N * f / F, hi = N * (f + 1) / F;
    float* pdq = pd + (qq * F + f) * k;
    int64_t* piq = pi + (qq * F + f) * k;
    exact_query_topk<DV>(tab, inv, lo, hi, qn + qq * DV * 4, k, dl, piq, pdq);
    if (!last_arriver(pcnt + qq, F, &last)) return;
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      float d = FLT_MAX;
      int i = INT_MAX;
      for (int ff = 0; ff < F; ++ff) {
        const int sl = ff == 0 ? lane : lane - k;
        if (ff == 0 || lane >= k) {
          const bool has = sl >= 0 && sl < k;
          const float dv = has ? pd[(qq * F + ff) * k + sl] : FLT_MAX;
          const int64_t iv = has ? pi[(qq * F + ff) * k + sl] : (int64_t)INT_MAX;
          d = dv;
          i = dv == FLT_MAX ? INT_MAX : (int)iv;   // (a range shorter than k: FLT_MAX / INT_MAX pads)
        }
        if (ff > 0) wave_sort64(d, i, lane);
      }
      if (lane < k) {
        idx[qq * k + lane] = (int64_t)i;
        dist[qq * k + lane] = d;
      }
    }
  };
  if (f > 0) {   // a split-fallback block: only for an overflowed list
    const int n = qcnt[qq];
    if (n > V4_CAP || n < k) split();
    return;
  }
  const int* rl = rows + qq * V4_CAP;
  const float* dq = dists + qq * V4_CAP;
  // the list's first B4_T entries are read beside its count (the slots
  // exist whatever the count; the ones past it are ignored): one round trip
  const float d0 = dq[threadIdx.x];
  const int i0 = rl[threadIdx.x];
  const int n = qcnt[qq];
  if (n > V4_CAP || n < k) {   // overflow (fewer than k admitted rows only when N < k)
    if (F > 1) split();
    else if (FB == 0) fail();
    else join_pool();   // (the pool answers it)
    return;
  }
  if (threadIdx.x == 0) cnt = 0;
  if ((int)threadIdx.x < n) dl[threadIdx.x] = d0;
  for (int e = threadIdx.x + B4_T; e < n; e += B4_T) dl[e] = dq[e];
  __syncthreads();
  const unsigned tk = block_select_kth<B4_T>(dl, n, k);   // upper edge of the k-th's bin
  for (int e = threadIdx.x; e < n; e += B4_T)
    if (__float_as_uint(dl[e]) <= tk) {
      const int pos = atomicAdd(&cnt, 1);
      cd[pos] = dl[e];
      ci[pos] = e < B4_T ? i0 : rl[e];
    }
  __syncthreads();
  // (many rows sharing the k-th's bin -- duplicates -- are sorted here too,
  // up to the whole list: round 5 sent a bin of more than 256 rows to the
  // exact table scan, 9.9 ms for 256 such queries over 1M rows)
  const int nv = cnt;
  if (nv <= 64) {   // (the usual case) one wave's register sort, no more barriers
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      float d = lane < nv ? cd[lane] : FLT_MAX;
      int i = lane < nv ? ci[lane] : INT_MAX;
      wave_sort64(d, i, lane);
      if (lane < k) {
        idx[qq * k + lane] = (int64_t)i;
        dist[qq * k + lane] = d;
      }
    }
    if (pool) join_pool();
    return;
  }
  int n2 = 2;
  while (n2 < nv) n2 <<= 1;
  for (int t = nv + threadIdx.x; t < n2; t += B4_T) { cd[t] = FLT_MAX; ci[t] = INT_MAX; }
  __syncthreads();
  bitonic<B4_T>(cd, ci, n2);
  for (int t = threadIdx.x; t < k; t += B4_T) {
    idx[qq * k + t] = (int64_t)ci[t];
    dist[qq * k + t] = cd[t];
  }
  if (pool) join_pool();
}

// Per query: the k best of nslices k-lists.  All of a chunk's candidates are
// loaded up front (MT per thread, one round trip), then filtered against the
// running k-th best and compacted in LDS.
constexpr int MT = 16;
constexpr int FT = 24;   // fast path: candidates loaded per thread per round
// groups > 1: block (query, group) merges lists [g*lpg, (g+1)*lpg) of its
// query into gout[query][group] (a first stage); groups == 1: the final
// stage writes idx / dist.
__global__ __launch_bounds__(NT) void merge_kernel(const Cand* in, int nslices, int k,
                                                   int64_t* idx, float* dist, int groups,
                                                   Cand* gout) {
  __shared__ float cd[CAP];
  __shared__ int ci[CAP];
  __shared__ int cnt;
  __shared__ float thr;
  const int64_t qq = blockIdx.x / groups;
  const int grp = blockIdx.x % groups;
  const int lpg = (nslices + groups - 1) / groups;
  const int l0 = grp * lpg, nl = max(0, min(lpg, nslices - l0));
  const Cand* c = in + (qq * (int64_t)nslices + l0) * k;
  const int total = nl * k;
  // fast path 0 (final stage, one load round, up to 4 lists per thread): the
  // k-th smallest of the lists' minima bounds the k-th best overall (k lists
  // each hold a candidate at or under it), so only the candidates at or under
  // that bound -- found by a 2-pass radix select over the minima -- are sorted.
  // Same result as sorting them all: every candidate of the k best passes.
  if (groups == 1 && total <= NT * FT && nl <= 4 * NT) {
    __shared__ unsigned hist[256];
    __shared__ unsigned sel_prefix, sel_need;
    __shared__ int sel_fail;
    Cand e[FT];
#pragma unroll
    for (int j = 0; j < FT; ++j) {
      const int t = j * NT + threadIdx.x;
      e[j] = t < total ? c[t] : Cand{FLT_MAX, INT_MAX};
    }
    // distances are >= 0: their bits order like the values
    auto key = [](float x) { return __float_as_uint(fmaxf(x, 0.f)); };
    unsigned mk[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int l = threadIdx.x + r * NT;
      float m = FLT_MAX;
      if (l < nl)
        for (int j = 0; j < k; ++j) m = fminf(m, c[(int64_t)l * k + j].d);
      mk[r] = l < nl ? key(m) : 0xffffffffu;
    }
    if (threadIdx.x == 0) { sel_prefix = 0; sel_need = (unsigned)k; sel_fail = 0; }
    unsigned mask = 0;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int sh = 24 - 8 * pass;
      for (int b = threadIdx.x; b < 256; b += NT) hist[b] = 0;
      __syncthreads();
      const unsigned prefix = sel_prefix;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (mk[r] != 0xffffffffu && (mk[r] & mask) == prefix) atomicAdd(&hist[(mk[r] >> sh) & 255u], 1u);
      __syncthreads();
      if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const unsigned need = sel_need;
        unsigned h[4], sum = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) { h[b] = hist[4 * lane + b]; sum += h[b]; }
        unsigned incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned v = __shfl_up(incl, off, 64);
          if (lane >= off) incl += v;
        }
        unsigned cum = incl - sum;
        if (cum < need && need <= incl) {
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            if (cum + h[b] >= need) {
              sel_prefix = prefix | ((unsigned)(4 * lane + b) << sh);
              sel_need = need - cum;
              break;
            }
            cum += h[b];
          }
        }
        if (lane == 63 && incl < need) sel_fail = 1;   // fewer than k lists hold candidates
      }
      mask |= 255u << sh;
      __syncthreads();
    }
    if (!sel_fail) {
      const unsigned tk = sel_prefix | 0xffffu;
      if (threadIdx.x == 0) cnt = 0;
      __syncthreads();
      constexpr int SCAP = 128;
#pragma unroll
      for (int j = 0; j < FT; ++j)
        if (e[j].i != INT_MAX && key(e[j].d) <= tk) {
          const int pos = atomicAdd(&cnt, 1);
          if (pos < SCAP) { cd[pos] = e[j].d; ci[pos] = e[j].i; }
        }
      __syncthreads();
      const int nv = cnt;
      if (nv <= SCAP) {
        int n2 = 2;
        while (n2 < nv) n2 <<= 1;
        for (int t = nv + threadIdx.x; t < n2; t += NT) { cd[t] = FLT_MAX; ci[t] = INT_MAX; }
        __syncthreads();
        bitonic(cd, ci, n2);
        for (int t = threadIdx.x; t < k; t += NT) {
          const bool ok = t < nv;
          idx[qq * k + t] = ok ? (int64_t)ci[t] : -1;
          dist[qq * k + t] = ok ? cd[t] : FLT_MAX;
        }
        return;
      }
    }
    __syncthreads();
  }
  // fast path: the valid candidates (with admission bounds, a few per query)
  // fit the buffer -> one gather and one sort
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (int base = 0; base < total; base += NT * FT) {
    Cand e[FT];   // all loads of a round in flight together
#pragma unroll
    for (int j = 0; j < FT; ++j) {
      const int t = base + j * NT + threadIdx.x;
      e[j] = t < total ? c[t] : Cand{FLT_MAX, INT_MAX};
    }
#pragma unroll
    for (int j = 0; j < FT; ++j)
      if (e[j].i != INT_MAX) {
        const int pos = atomicAdd(&cnt, 1);
        if (pos < CAP) { cd[pos] = e[j].d; ci[pos] = e[j].i; }
      }
  }
  __syncthreads();
  const int nv = cnt;
  if (nv <= CAP) {
    int n2 = 2;
    while (n2 < nv) n2 <<= 1;
    for (int t = nv + threadIdx.x; t < n2; t += NT) { cd[t] = FLT_MAX; ci[t] = INT_MAX; }
    __syncthreads();
    bitonic(cd, ci, n2);
    for (int t = threadIdx.x; t < k; t += NT) {
      const bool ok = t < nv;
      if (groups > 1) {
        gout[(qq * groups + grp) * k + t] = Cand{ok ? cd[t] : FLT_MAX, ok ? ci[t] : INT_MAX};
      } else {
        idx[qq * k + t] = ok ? (int64_t)ci[t] : -1;
        dist[qq * k + t] = ok ? cd[t] : FLT_MAX;
      }
    }
    return;
  }
  __syncthreads();
  if (threadIdx.x == 0) { cnt = 0; thr = FLT_MAX; }
  __syncthreads();
  for (int base = 0; base < total; base += NT * MT) {
    Cand e[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int t = base + j * NT + threadIdx.x;
      e[j] = t < total ? c[t] : Cand{FLT_MAX, INT_MAX};
    }
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      if (e[j].i != INT_MAX && e[j].d <= thr) {
        int pos = atomicAdd(&cnt, 1);
        cd[pos] = e[j].d;
        ci[pos] = e[j].i;
      }
      __syncthreads();
      if (cnt > CAP - NT) compact(cd, ci, &cnt, &thr, k);
    }
  }
  compact(cd, ci, &cnt, &thr, k);
  for (int t = threadIdx.x; t < k; t += NT) {
    bool ok = t < cnt;
    if (groups > 1) {
      gout[(qq * groups + grp) * k + t] = Cand{ok ? cd[t] : FLT_MAX, ok ? ci[t] : INT_MAX};
    } else {
      idx[qq * k + t] = ok ? (int64_t)ci[t] : -1;
      dist[qq * k + t] = ok ? cd[t] : FLT_MAX;
    }
  }
}

// Per query: the k best of `lists` k-lists [lists][Q][k] (dist, int64 row),
// ascending by (dist, row as unsigned); padding entries (FLT_MAX, -1) sort
// last.  One block per query, all lists*k <= TM_CAP candidates sorted in LDS.
constexpr int TM_CAP = 2048;
__global__ __launch_bounds__(NT) void topk_merge_kernel(const float* dist, const int64_t* idx,
                                                        int lists, int64_t Q, int k,
                                                        int64_t* out_idx, float* out_dist) {
  __shared__ float cd[TM_CAP];
  __shared__ uint64_t ci[TM_CAP];
  const int64_t qq = blockIdx.x;
  const int n = lists * k;
  int n2 = 2;
  while (n2 < n) n2 <<= 1;
  for (int t = threadIdx.x; t < n2; t += NT) {
    if (t < n) {
      const int64_t src = ((int64_t)(t / k) * Q + qq) * k + t % k;
      cd[t] = dist[src];
      ci[t] = (uint64_t)idx[src];
    } else {
      cd[t] = FLT_MAX;
      ci[t] = ~0ull;
    }
  }
  __syncthreads();
  for (int k2 = 2; k2 <= n2; k2 <<= 1) {
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += NT) {
        const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
        const int p = i + j;
        const bool asc = (i & k2) == 0;
        const float a = cd[i], b = cd[p];
        const uint64_t ia = ci[i], ib = ci[p];
        const bool bl = b < a || (b == a && ib < ia);
        const bool al = a < b || (a == b && ia < ib);
        if (asc ? bl : al) { cd[i] = b; cd[p] = a; ci[i] = ib; ci[p] = ia; }
      }
      __syncthreads();
    }
  }
  for (int t = threadIdx.x; t < k; t += NT) {
    out_idx[qq * k + t] = (int64_t)ci[t];
    out_dist[qq * k + t] = cd[t];
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

// The fit-time bf16 copy read by scan v4: out[r][c] = bf16(t[r][c] * inv[r])
// (fp32 product, round to nearest even -- the rounding scan v4 otherwise
// applies to the fp32 rows on the fly).  8 elements per thread, d % 8 == 0.
__global__ void pack_rows_kernel(const float* __restrict__ t, const float* __restrict__ inv, int64_t N, int d,
                                 bf16* __restrict__ out) {
  const int64_t n8 = N * d / 8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    const float iv = inv[e * 8 / d];
    const float4 u = reinterpret_cast<const float4*>(t)[2 * e], v = reinterpret_cast<const float4*>(t)[2 * e + 1];
    reinterpret_cast<bf16x8*>(out)[e] = bf16x8{(bf16)(u.x * iv), (bf16)(u.y * iv), (bf16)(u.z * iv), (bf16)(u.w * iv),
                                               (bf16)(v.x * iv), (bf16)(v.y * iv), (bf16)(v.z * iv), (bf16)(v.w * iv)};
  }
}

}  // namespace

dcnr_status row_inv_norms(const float* t, int64_t N, int d, float* out, hipStream_t s) {
  if (N <= 0) return DCNR_OK;
  int64_t blocks = std::min<int64_t>(cdiv(N, 4), 8192);
  hipLaunchKernelGGL(inv_norm_kernel, dim3((unsigned)blocks), dim3(256), 0, s, t, N, d, out);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status cosine_pack_rows(const float* t, const float* inv, int64_t N, int d, bf16* out, hipStream_t s) {
  if (d % 8) {
    set_error("cosine_pack_rows: d=%d is not a multiple of 8", d);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (N <= 0) return DCNR_OK;
  const int64_t blocks = std::min<int64_t>(cdiv(N * d / 8, 256), 8192);
  hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, t, inv, N, d, out);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

bool use_v2(int d, int k) { return d % 4 == 0 && d >= 4 && d <= 64 && k <= K2_KMAX; }

// v2 plan: up to 512 row slices (2 blocks per CU per query tile), slices a
// multiple of 64 rows
void plan2(int64_t N, int* nslices, int64_t* rows_per_block) {
  const int64_t want = std::min<int64_t>(512, std::max<int64_t>(1, cdiv(N, 256)));
  *rows_per_block = rup(cdiv(N, want), 64);
  *nslices = (int)cdiv(N, *rows_per_block);
}

bool use_v4(int64_t N, int64_t Q, int d, int k) {
  // Any table size: one of at most V4_S rows is its own sample (pass 1 is
  // then the whole search).  A single query over fewer than V4_Q1_N rows takes scan
  // v2, whose one pass beats v4's fixed chain (29 vs 50 us at 20000 rows, 65
  // vs 61 at 1M); v4's exact distances use v2's arithmetic, so the choice
  // never changes an answer.
  return use_v2(d, k) && Q >= 1 && d % 32 == 0 && (Q > 1 || N >= V4_Q1_N);
}

// v4 scratch after the v2 layout (cands | qn [Q][d] | thr0 [Q]): bf16
// queries [Q][d] | per-query counts [Q] | admitted rows [Q][V4_CAP]
// | their exact distances [Q][V4_CAP] | the bound's block minima
// [Q][B5_G]
// the split fallback's k-lists (k <= 32: scan v4's range), for Q <= V4_FQ
size_t v4_split_bytes(int64_t Q) {
  const int L = v4_lists(Q);
  return L > 1 ? rup((size_t)Q * L * 32 * 4, 256) + (size_t)Q * L * 32 * 8 : 0;
}
size_t v4_extra(int64_t Q, int d) {
  return rup((size_t)Q * d * 2, 256) + rup((size_t)Q * 8 + 48, 256) + 2 * (size_t)Q * V4_CAP * 4 +
         rup((size_t)Q * B5_G * 4, 256) + v4_split_bytes(Q) + 256;
}

size_t topk_ws_d(int64_t N, int64_t Q, int k, int d) {
  int ns; int64_t rps;
  if (use_v2(d, k)) {
    plan2(N, &ns, &rps);
    const size_t v2 = rup((size_t)Q * ns * k * sizeof(Cand), 256) + (size_t)Q * (d + 1) * 4;
    return use_v4(N, Q, d, k) ? rup(v2, 256) + v4_extra(Q, d) : v2;
  }
  plan(N, Q, k, &ns, &rps);
  return (size_t)Q * ns * k * sizeof(Cand);
}

// Final merge of the per-block k-lists, one block per query.  Measured at
// 1M rows (512 lists, 5632 candidates per query): this filter-and-compact
// block 32 us; a two-stage (16 groups, then the group lists) 32 + 16 us; a
// one-shot 8192-entry bitonic sort by 1024 threads 107 us; a per-wave register
// merge 50 us -- the block barriers of a one-block kernel dominate all of them.
dcnr_status merge_lists(const Cand* cands, int64_t Q, int ns, int k, int64_t* idx, float* dist,
                        hipStream_t s) {
  hipLaunchKernelGGL(merge_kernel, dim3((unsigned)Q), dim3(NT), 0, s, cands, ns, k, idx, dist, 1,
                     nullptr);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

// enough for every d (the v2 path keeps Q x d <= Q x 64 normalised queries)
size_t topk_ws(int64_t N, int64_t Q, int k) {
  int ns; int64_t rps;
  plan(N, Q, k, &ns, &rps);
  return std::max(topk_ws_d(N, Q, k, 64), (size_t)Q * ns * k * sizeof(Cand));
}

dcnr_status cosine_topk(const float* t, const float* inv, const bf16* tb, int64_t N, int d,
                        const float* q, int64_t Q, int k, int64_t* idx, float* dist, void* ws,
                        size_t ws_bytes, hipStream_t s) {
  if (k < 1 || k > KMAX || d < 4 || d % 4 || d > 256 || N < 1) {
    set_error("cosine_topk: unsupported k=%d d=%d N=%lld (1<=k<=64, d%%4==0, d<=256)", k, d,
              (long long)N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (Q <= 0) return DCNR_OK;
  if (ws_bytes < topk_ws_d(N, Q, k, d)) {
    set_error("cosine_topk: workspace too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  int ns; int64_t rps;
  Cand* cands = (Cand*)ws;
  if (use_v2(d, k)) {
    plan2(N, &ns, &rps);
    float* qn = (float*)((char*)ws + rup((size_t)Q * ns * k * sizeof(Cand), 256));
    // normalised queries + admission bounds, one block per query (v4 makes
    // its own, from a larger sample, below)
    float* thr0 = qn + Q * d;
    const bool v4 = use_v4(N, Q, d, k);
    bf16* qb = nullptr;
    int *qcnt = nullptr, *rows = nullptr;   // v4 scratch
    float* dists = nullptr;
    float* bmins = nullptr;             // v4 bound: block minima
    float* split_d = nullptr;           // v4 split fallback: k-lists
    int64_t* split_i = nullptr;
    if (v4) {
      char* x = (char*)ws + rup(rup((size_t)Q * ns * k * sizeof(Cand), 256) + (size_t)Q * (d + 1) * 4, 256);
      qb = (bf16*)x;
      x += rup((size_t)Q * d * 2, 256);
      qcnt = (int*)x;   // [Q] list counts, the overflow word, [Q] fallback arrival counters,
                        // a spare word, the batched fallback's 8 queue heads
      x += rup((size_t)Q * 8 + 48, 256);
      rows = (int*)x;
      dists = (float*)(rows + Q * V4_CAP);
      x += 2 * (size_t)Q * V4_CAP * 4;
      bmins = (float*)x;
      x += rup((size_t)Q * B5_G * 4, 256);
      split_d = (float*)x;
      split_i = (int64_t*)(x + rup((size_t)Q * v4_lists(Q) * 32 * 4, 256));
    }
    if (!v4) {
      switch (d / 4) {
#define CASEK(n)                                                                             \
  case n:                                                                                    \
    hipLaunchKernelGGL(kth_bound_kernel<n>, dim3((unsigned)Q), dim3(256), 0, s, t, inv, N, q, qn, k, \
                       thr0);                                                                          \
    break;
        CASEK(1) CASEK(2) CASEK(3) CASEK(4) CASEK(5) CASEK(6) CASEK(7) CASEK(8)
        CASEK(9) CASEK(10) CASEK(11) CASEK(12) CASEK(13) CASEK(14) CASEK(15) CASEK(16)
#undef CASEK
      }
      DCNR_LAUNCH_CHECK();
    }
    if (v4) {
      // query blocks of 16: NQB per launch row (the table is read once per
      // NQB * 16 queries)
      const int nqb = (int)std::min<int64_t>(cdiv(Q, 16), V4_QC / 16);
      const int NQ = nqb <= 2 ? 2 : nqb <= 4 ? 4 : nqb <= 8 ? 8 : 16;
      const int rpb = v4_rpb(NQ, N);
      const dim3 g4((unsigned)cdiv(N, rpb), (unsigned)cdiv(Q, NQ * 16));
      // the admission bound from the first V4_S rows (bound5_kernel), its
      // minima merged by scan4 itself up to V4_MQ queries
      const int ng = (int)cdiv(std::min<int64_t>(N, V4_S), B5_C);
      const bool merge4 = Q <= V4_MQ;
      {
        const int qg = merge4 ? 1 : B5_QG;
        const dim3 gb((unsigned)ng, (unsigned)cdiv(Q, 16 * qg));
#define BOUND5(ks, pk)                                                                                         \
  do {                                                                                                         \
    if (merge4)                                                                                                \
      hipLaunchKernelGGL((bound5_kernel<ks, pk, 1>), gb, dim3(256), 0, s, t, inv, tb, N, q, Q, qn, qb, qcnt, bmins); \
    else                                                                                                       \
      hipLaunchKernelGGL((bound5_kernel<ks, pk, B5_QG>), gb, dim3(256), 0, s, t, inv, tb, N, q, Q, qn, qb, qcnt,     \
                         bmins);                                                                               \
  } while (0)
        if (d == 32) {
          if (tb) BOUND5(1, true);
          else BOUND5(1, false);
        } else {
          if (tb) BOUND5(2, true);
          else BOUND5(2, false);
        }
#undef BOUND5
        DCNR_LAUNCH_CHECK();
        if (!merge4) {
          hipLaunchKernelGGL(bound5_merge_kernel, dim3((unsigned)cdiv(Q, 4)), dim3(256), 0, s, bmins, ng, Q, k,
                             thr0);
          DCNR_LAUNCH_CHECK();
        }
      }
#define SCAN4(ks, nq, pk, g, n, rp)                                                                    \
  hipLaunchKernelGGL((scan4_kernel<ks, nq, pk>), g, dim3(256), 0, s, t, inv, tb, n, rp, qb, thr0, qn, \
                     Q, qcnt, rows, dists, merge4 ? bmins : nullptr, ng, k)
#define CASE4(ks, nq, sel, g, n, rp)                                  \
  if (d == 32 * ks && sel == nq) {                                    \
    if (tb) SCAN4(ks, nq, true, g, n, rp);                            \
    else SCAN4(ks, nq, false, g, n, rp);                              \
  }
#define CASES4(sel, g, n, rp)                                                             \
  CASE4(1, 2, sel, g, n, rp) CASE4(1, 4, sel, g, n, rp) CASE4(1, 8, sel, g, n, rp)         \
  CASE4(1, 16, sel, g, n, rp) CASE4(2, 2, sel, g, n, rp) CASE4(2, 4, sel, g, n, rp)        \
  CASE4(2, 8, sel, g, n, rp) CASE4(2, 16, sel, g, n, rp)
      CASES4(NQ, g4, N, rpb)
      DCNR_LAUNCH_CHECK();
      // (a query whose list overflowed: the split fallback for Q <= V4_FQ,
      // else the batched fallback's pool, inside these blocks)
      const int F = v4_fallback_split(Q);
      const int FB = v4_batch_chunks(Q);
      const unsigned nb = (unsigned)(Q * F);
      if (d == 32)
        hipLaunchKernelGGL(rescore_kernel<8>, dim3(nb), dim3(B4_T), 0, s, dists, qcnt, rows, k,
                           idx, dist, t, inv, N, qn, Q, F, FB, split_d, split_i, qcnt + Q + 1);
      else
        hipLaunchKernelGGL(rescore_kernel<16>, dim3(nb), dim3(B4_T), 0, s, dists, qcnt, rows, k,
                           idx, dist, t, inv, N, qn, Q, F, FB, split_d, split_i, qcnt + Q + 1);
      DCNR_LAUNCH_CHECK();
#undef CASES4
#undef CASE4
#undef SCAN4
      return DCNR_OK;
    }
    if (!v4 && Q >= MFMA_MIN_Q && d % 16 == 0) {
      const int qtiles = (int)cdiv(Q, K3_QT);
      const int64_t blocks = rup(ns, 8) * qtiles;
      switch (d / 16) {
#define CASE3(n)                                                                                   \
  case n:                                                                                          \
    hipLaunchKernelGGL(scan3_kernel<4 * n>, dim3((unsigned)blocks), dim3(K2_NT), 0, s, t, inv, N,  \
                       qn, Q, k, rps, ns, qtiles, cands, thr0);                              \
    break;
        CASE3(1) CASE3(2) CASE3(3) CASE3(4)
#undef CASE3
      }
      DCNR_LAUNCH_CHECK();
      return merge_lists(cands, Q, ns, k, idx, dist, s);
    }
    // scan v2: the exact VALU scan (the same distance arithmetic as v4's
    // rescoring and its per-query fallback)
    const int qtiles = (int)cdiv(Q, K2_QT);
    const int64_t blocks = rup(ns, 8) * qtiles;
    switch (d / 4) {
#define CASE(n)                                                                                  \
  case n:                                                                                        \
    hipLaunchKernelGGL(scan2_kernel<n>, dim3((unsigned)blocks), dim3(K2_NT), 0, s, t, inv, N, qn, \
                       Q, k, rps, ns, qtiles, cands, thr0);                                \
    break;
      CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
      CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    }
    DCNR_LAUNCH_CHECK();
    return merge_lists(cands, Q, ns, k, idx, dist, s);
  }
  plan(N, Q, k, &ns, &rps);
  dim3 grid(ns, (unsigned)cdiv(Q, QT));
  if (d <= 64)
    hipLaunchKernelGGL(scan_kernel<16>, grid, dim3(NT), 0, s, t, inv, N, d, q, Q, k, rps, cands);
  else
    hipLaunchKernelGGL(scan_kernel<64>, grid, dim3(NT), 0, s, t, inv, N, d, q, Q, k, rps, cands);
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(merge_kernel, dim3((unsigned)Q), dim3(NT), 0, s, cands, ns, k, idx, dist, 1,
                     nullptr);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status topk_merge(const float* dist, const int64_t* idx, int lists, int64_t Q, int k,
                       int64_t* out_idx, float* out_dist, hipStream_t s) {
  if (k < 1 || lists < 1 || (int64_t)lists * k > TM_CAP) {
    set_error("topk_merge: %d lists of k=%d unsupported (lists * k <= %d)", lists, k, TM_CAP);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (Q <= 0) return DCNR_OK;
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)Q), dim3(NT), 0, s, dist, idx, lists, Q, k,
                     out_idx, out_dist);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
