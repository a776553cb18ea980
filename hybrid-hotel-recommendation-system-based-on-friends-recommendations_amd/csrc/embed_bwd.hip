// Deterministic dense embedding gradients: the embedding_dense_backward that
// loss.backward() runs for every nn.Embedding of DCN_RecSys (reference
// train.py:156-158 embeddings, :225 backward; dense grads, sparse=False).
//
// grad_t[r] = sum over samples b with id_t[b] == r of dx0[b, off_t : off_t+w_t]
//
// in a FIXED order (ascending b within a run), so two runs on the same
// inputs give bit-identical gradients (the fp32 scatter-atomics they replace
// did not).  Three steps per step of the backward:
//
//   1. emb_keys_kernel: key = base_t + id (all tables in one key space),
//      value = b, laid out table-major: entries of table t at [t*B, (t+1)*B).
//   2. rocPRIM radix_sort_pairs (stable): after it table t still occupies
//      [t*B, (t+1)*B) (its keys lie in [base_t, base_t + rows_t)) and each
//      run of equal keys lists its samples in ascending b.  Steps 1-2 read
//      only the ids, so dcnr_backward runs them on a side stream while the
//      deep-tower backward runs (they join before step 3).
//   3. emb_runs_short_kernel: the thread at a run's head sums runs of <= LIM
//      entries sequentially and writes the row; emb_runs_long_kernel: the
//      wave whose 64 positions hold the head of a longer run (popular ids,
//      small categorical tables) reduces it (entries strided over lane
//      slots, slots combined in fixed lane order).  No global counters or
//      lists: a device-scope atomic per long run (12000 at the bench size)
//      serialised at memory and cost ~100 us.
//
// Step 3 reads dx0_total (written by the cross backward: cross part + deep
// part of each table's columns, table-major so that an entry's w_t floats are
// one aligned segment -- in the row-major [B][Dp] dx0 three in four 128-B
// segments straddled two lines) once per entry: 4*w_t + 8 bytes per
// (sample, table) + one row write per distinct id.
#include "dcnr_internal.h"

#include <cstring>
#include <mutex>
#include <rocprim/device/device_radix_sort.hpp>

namespace dcnr {
namespace {

constexpr int ENT = 256;          // threads per block
constexpr int LIM = 16;           // longest run the short kernel sums in one thread

struct EmbTabs {
  float* grad[MAX_TABLES];
  uint32_t base[MAX_TABLES];
  int64_t rows[MAX_TABLES];
  int width[MAX_TABLES];
  int off[MAX_TABLES];
};

EmbTabs make_tabs(const EmbBwdDesc& e) {
  EmbTabs t;
  memset(&t, 0, sizeof(t));
  uint32_t base = 0;
  for (int i = 0; i < e.n_tab; ++i) {
    t.grad[i] = e.grad[i];
    t.base[i] = base;
    t.rows[i] = e.rows[i];
    t.width[i] = e.width[i];
    t.off[i] = e.off[i];
    base += (uint32_t)e.rows[i];
  }
  return t;
}

int key_bits(const EmbBwdDesc& e) {
  uint64_t total = 0;
  for (int i = 0; i < e.n_tab; ++i) total += (uint64_t)e.rows[i];
  int bits = 1;
  while (bits < 32 && (1ull << bits) < total) ++bits;
  return bits;
}

__global__ __launch_bounds__(ENT) void emb_keys_kernel(EmbTabs et, int nt, const int64_t* user,
                                                       const int64_t* item, const int64_t* cat,
                                                       int64_t B, uint32_t* keys, uint32_t* vals) {
  const int64_t i = (int64_t)blockIdx.x * ENT + threadIdx.x;
  if (i >= (int64_t)nt * B) return;
  const int t = (int)(i / B);
  const int64_t b = i - (int64_t)t * B;
  int64_t id = t == 0 ? user[b] : t == 1 ? item[b] : cat[b * (nt - 2) + (t - 2)];
  const int64_t rows = et.rows[t];
  id = id < 0 ? 0 : (id >= rows ? rows - 1 : id);   // the forward gather's clamp
  keys[i] = et.base[t] + (uint32_t)id;
  vals[i] = (uint32_t)b;
}

template <int VEC> struct Vec;
template <> struct Vec<1> {
  typedef float T;
  static __device__ __forceinline__ T ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, T v) { *p = v; }
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T shfl(T v, int src) { return __shfl(v, src); }
};
template <> struct Vec<4> {
  typedef f32x4 T;
  static __device__ __forceinline__ T ld(const float* p) { return *reinterpret_cast<const T*>(p); }
  static __device__ __forceinline__ void st(float* p, T v) { *reinterpret_cast<T*>(p) = v; }
  static __device__ __forceinline__ T zero() { return T{0.f, 0.f, 0.f, 0.f}; }
  static __device__ __forceinline__ T shfl(T v, int src) {
    return T{__shfl(v[0], src), __shfl(v[1], src), __shfl(v[2], src), __shfl(v[3], src)};
  }
};

// One thread per sorted position; the head of a run of <= LIM entries sums
// it in ascending sample order.  Latency, not bandwidth, bounds this kernel
// (a few KB per wave, scattered rows), so no load waits on another it does
// not depend on: the run's keys and samples are loaded together, and its dx0
// rows EG entries at a time (UNR column groups of VEC per pass).
template <int VEC>
__global__ __launch_bounds__(ENT) void emb_runs_short_kernel(EmbTabs et, int nt, int64_t B,
                                                             const uint32_t* ks,
                                                             const uint32_t* vs,
                                                             const float* dx0, int accumulate) {
  typedef Vec<VEC> V;
  typedef typename V::T T;
  constexpr int UNR = 16 / VEC;   // 16 columns per pass
  constexpr int EG = 4;           // entries whose loads are in flight together
  const int64_t i = (int64_t)blockIdx.x * ENT + threadIdx.x;
  if (i >= (int64_t)nt * B) return;
  const int t = (int)(i / B);
  const int64_t t0 = (int64_t)t * B, t1 = t0 + B;
  const uint32_t k = ks[i];
  if (i > t0 && ks[i - 1] == k) return;   // not the head of its run
  uint32_t nk[LIM];
#pragma unroll
  for (int q = 0; q < LIM; ++q) nk[q] = i + 1 + q < t1 ? ks[i + 1 + q] : ~0u;
  if (nk[LIM - 1] == k) return;   // longer than LIM (keys are sorted): the long kernel's
  int len = 1;
#pragma unroll
  for (int q = 0; q < LIM - 1; ++q) len += nk[q] == k;
  uint32_t smp[LIM];
#pragma unroll
  for (int q = 0; q < LIM; ++q) smp[q] = q < len ? vs[i + q] : 0u;
  const int w = et.width[t];
  const float* src = dx0 + B * et.off[t];   // table t's [B][w] block
  float* dst = et.grad[t] + (int64_t)(k - et.base[t]) * w;
  for (int c = 0; c < w; c += UNR * VEC) {
    T acc[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc[u] = V::zero();
#pragma unroll
    for (int q0 = 0; q0 < LIM; q0 += EG) {
      if (q0 >= len) break;
      T x[EG][UNR];
#pragma unroll
      for (int q = 0; q < EG; ++q) {
        const float* row = src + (int64_t)smp[q0 + q] * w + c;
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          x[q][u] = (q0 + q < len && c + u * VEC < w) ? V::ld(row + u * VEC) : V::zero();
      }
#pragma unroll
      for (int q = 0; q < EG; ++q)
        if (q0 + q < len)
#pragma unroll
          for (int u = 0; u < UNR; ++u) acc[u] += x[q][u];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (c + u * VEC < w) {
        float* p = dst + c + u * VEC;
        V::st(p, accumulate ? V::ld(p) + acc[u] : acc[u]);
      }
  }
}

// One wave per long run, walked WAVE entries at a time: lane L holds entry
// p+L's key and sample (coalesced loads, the next block's issued before this
// block's dx0 rows), the column groups of VEC sit across lanes and the
// block's entries across the remaining S = 64/Gb lane slots (slot s takes
// entries s, s+S, ... of every block, summing them in ascending order),
// slots added in ascending order at the end.  The wave owning the run's
// head position (64 positions per wave) reduces it.
template <int VEC>
__global__ __launch_bounds__(ENT) void emb_runs_long_kernel(EmbTabs et, int64_t B, int64_t n,
                                                            const uint32_t* ks,
                                                            const uint32_t* vs,
                                                            const float* dx0, int accumulate) {
  typedef Vec<VEC> V;
  typedef typename V::T T;
  constexpr int QMAX = 8;   // entries per slot per block held in flight (S >= 8)
  const int lane = threadIdx.x & 63;
  // this wave's 64 positions: which start a run longer than LIM
  const int64_t base = ((int64_t)blockIdx.x * (ENT / WAVE) + (threadIdx.x >> 6)) * WAVE;
  bool head = false;
  {
    const int64_t i = base + lane;
    if (i < n) {
      const int t = (int)(i / B);
      const int64_t t0 = (int64_t)t * B;
      const uint32_t k = ks[i];
      head = (i == t0 || ks[i - 1] != k) && i + LIM < t0 + B && ks[i + LIM] == k;
    }
  }
  for (uint64_t hm = __ballot(head); hm; hm &= hm - 1) {
    const int64_t i = base + __builtin_ctzll(hm);
    const uint32_t k = ks[i];
    const int t = (int)(i / B);
    const int64_t t1 = (int64_t)(t + 1) * B;
    const int w = et.width[t], G = w / VEC;
    const float* src = dx0 + B * et.off[t];   // table t's [B][w] block
    float* dst = et.grad[t] + (int64_t)(k - et.base[t]) * w;
    for (int cb = 0; cb < G; cb += WAVE) {
      const int Gb = G - cb < WAVE ? G - cb : WAVE;
      const int S = WAVE / Gb, slot = lane / Gb, cg = lane - slot * Gb;
      const int col = (cb + cg) * VEC;
      const bool act = slot < S;
      T acc = V::zero();
      int64_t p = i;
      uint32_t kn = p + lane < t1 ? ks[p + lane] : ~0u;
      uint32_t sn = p + lane < t1 ? vs[p + lane] : 0u;
      for (;;) {
        const int nb = __popcll(__ballot(kn == k));   // the run's entries in this block: a prefix
        const int smp = (int)sn;
        const int64_t pn = p + WAVE;
        if (nb == WAVE) {   // the run may go on: fetch the next block now
          kn = pn + lane < t1 ? ks[pn + lane] : ~0u;
          sn = pn + lane < t1 ? vs[pn + lane] : 0u;
        }
        T x[QMAX];
#pragma unroll
        for (int q = 0; q < QMAX; ++q) {
          const int j = slot + S * q;
          const int b = __shfl(smp, j & 63);
          x[q] = (act && j < nb) ? V::ld(src + (int64_t)b * w + col) : V::zero();
        }
#pragma unroll
        for (int q = 0; q < QMAX; ++q)
          if (act && slot + S * q < nb) acc += x[q];
        for (int q = QMAX; S * q < WAVE; ++q) {   // S < 8 only; uniform trip count
          const int j = slot + S * q;
          const int b = __shfl(smp, j & 63);
          if (act && j < nb) acc += V::ld(src + (int64_t)b * w + col);
        }
        if (nb < WAVE) break;
        p = pn;
      }
      T tot = acc;
      for (int s = 1; s < S; ++s) {   // wave-uniform trip count
        const T v = V::shfl(acc, (s * Gb + cg) & 63);
        if (slot == 0) tot += v;
      }
      if (slot == 0) {
        float* q = dst + col;
        V::st(q, accumulate ? V::ld(q) + tot : tot);
      }
    }
  }
}

bool vec4_ok(const EmbBwdDesc& e, const float* dx0) {
  if ((uintptr_t)dx0 & 15) return false;
  for (int t = 0; t < e.n_tab; ++t)
    if (e.width[t] % 4 || e.off[t] % 4 || ((uintptr_t)e.grad[t] & 15)) return false;
  return true;
}

}  // namespace

size_t emb_sort_tmp_bytes(int64_t n) {
  // rocPRIM's own double buffer (8 B per pair) plus its histograms and
  // look-back state; dcnr_backward checks the library's exact figure
  return (size_t)n * 8 + (size_t)n / 4 + ((size_t)1 << 20);
}

dcnr_status emb_sort(const EmbBwdDesc& e, const int64_t* user, const int64_t* item,
                     const int64_t* cat, int64_t B, const EmbSortBufs& sb, hipStream_t s) {
  const int64_t n = (int64_t)e.n_tab * B;
  if (n <= 0) return DCNR_OK;
  uint64_t total = 0;
  for (int i = 0; i < e.n_tab; ++i) total += (uint64_t)e.rows[i];
  if (total >= (1ull << 32) || B >= (1ll << 32) || n >= (1ll << 31)) {
    set_error("embedding backward: %llu table rows / B=%lld beyond 32-bit keys",
              (unsigned long long)total, (long long)B);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  const EmbTabs et = make_tabs(e);
  hipLaunchKernelGGL(emb_keys_kernel, dim3((unsigned)cdiv(n, ENT)), dim3(ENT), 0, s, et, e.n_tab,
                     user, item, cat, B, sb.keys, sb.vals);
  DCNR_LAUNCH_CHECK();
  size_t need = 0;
  DCNR_HIP(rocprim::radix_sort_pairs(nullptr, need, sb.keys, sb.keys_s, sb.vals, sb.vals_s,
                                     (size_t)n, 0, key_bits(e), s));
  if (need > sb.tmp_bytes) {
    set_error("embedding backward: sort scratch %zu > reserved %zu", need, sb.tmp_bytes);
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  size_t have = sb.tmp_bytes;
  DCNR_HIP(rocprim::radix_sort_pairs(sb.tmp, have, sb.keys, sb.keys_s, sb.vals, sb.vals_s,
                                     (size_t)n, 0, key_bits(e), s));
  return DCNR_OK;
}

dcnr_status emb_segment_sum(const EmbBwdDesc& e, const EmbSortBufs& sb, int64_t B,
                            const float* dx0, int accumulate, hipStream_t s) {
  const int64_t n = (int64_t)e.n_tab * B;
  if (n <= 0) return DCNR_OK;
  const EmbTabs et = make_tabs(e);
  const dim3 gs((unsigned)cdiv(n, ENT));
  if (vec4_ok(e, dx0)) {
    hipLaunchKernelGGL(emb_runs_short_kernel<4>, gs, dim3(ENT), 0, s, et, e.n_tab, B, sb.keys_s,
                       sb.vals_s, dx0, accumulate);
    DCNR_LAUNCH_CHECK();
    hipLaunchKernelGGL(emb_runs_long_kernel<4>, gs, dim3(ENT), 0, s, et, B, n, sb.keys_s,
                       sb.vals_s, dx0, accumulate);
  } else {
    hipLaunchKernelGGL(emb_runs_short_kernel<1>, gs, dim3(ENT), 0, s, et, e.n_tab, B, sb.keys_s,
                       sb.vals_s, dx0, accumulate);
    DCNR_LAUNCH_CHECK();
    hipLaunchKernelGGL(emb_runs_long_kernel<1>, gs, dim3(ENT), 0, s, et, B, n, sb.keys_s,
                       sb.vals_s, dx0, accumulate);
  }
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

// Side stream for the id sort, one per device, created on first use.
dcnr_status emb_side_stream(hipStream_t* out) {
  static std::mutex mu;
  static hipStream_t streams[64] = {};
  int dev = 0;
  DCNR_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) {
    set_error("embedding backward: device %d out of range", dev);
    return DCNR_BAD_ARG;
  }
  std::lock_guard<std::mutex> lk(mu);
  if (!streams[dev]) DCNR_HIP(hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking));
  *out = streams[dev];
  return DCNR_OK;
}

}  // namespace dcnr
