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
//   1-2. a stable two-level counting sort of each table's (id, sample)
//      pairs (below: bucket counts per chunk, a scan, a stable scatter, then
//      per-bucket sorts on the low id bits); after it table t occupies
//      [t*B, (t+1)*B) of the sorted arrays (key = base_t + id) and each run
//      of equal keys lists its samples in ascending b.  (rocPRIM's
//      radix_sort_pairs did the same in ~107 us at the bench size: three
//      look-back-bound 8-bit passes.)
//   3. emb_runs_short_kernel: the thread at a run's head sums runs of <= LIM
//      entries sequentially and writes the row; emb_runs_long_kernel: the
//      wave whose 64 positions hold the head of a longer run (popular ids,
//      small categorical tables) reduces it (entries strided over lane
//      slots, slots combined in fixed lane order).  Runs of more than HSEG
//      entries are cut at the global HSEG-position grid: one wave per
//      segment sums its pieces (long kernel), the wave of the segment where
//      the run starts adds them in order (short kernel).  No global counters
//      or lists: a device-scope atomic per long run (12000 at the bench size)
//      serialised at memory and cost ~100 us.
//
// Step 3 reads, per (sample, table) entry, the table's segment of the deep
// dx0 (rows of Dq = 32-float multiples, so a 32-wide segment is one aligned
// 128-B line) and the sample's L+1 cross coefficients (cross_bwd.hip), and
// writes row = deep sum + sum_k coefficient sum_k V_k once per distinct id:
// 4*w_t + 4*(L+1) + 8 bytes per entry.
#include "dcnr_internal.h"

#include <cstring>
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

namespace dcnr {
namespace {

constexpr int ENT = 256;          // threads per block
// longest run the short kernel sums in one thread (8 / 32 measured the same
// per step; the tests' bit-exact emulation is written for 16)
constexpr int LIM = 16;

struct EmbTabs {
  float* grad[MAX_TABLES];
  uint32_t base[MAX_TABLES];
  int64_t rows[MAX_TABLES];
  int width[MAX_TABLES];
  int off[MAX_TABLES];
  const float* V[8];   // dx0_cross basis (w_0..w_{L-1}, w_f[H:]), indexed by x0 column
  uint8_t* touched;    // DCNR_FLAG_ROW_MAP: byte per key, 1 for every row written
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
  for (int k = 0; k < e.nv && k < 8; ++k) t.V[k] = e.V[k];
  t.touched = e.touched;
  return t;
}

// ------------------------------------------------------------ id sort
// Stable two-level counting sort of each table's (id, sample) pairs, table t
// landing in [t*B, (t+1)*B) of keys_s/vals_s (key = base_t + id) in
// ascending (id, sample) order -- no global atomics, no look-back chains:
//   level 1, by bucket = id >> sh_t (<= 4096 buckets per table):
//     emb_hist_kernel    per (table, chunk of CH samples) bucket counts (LDS)
//     emb_scan_kernel    per table, exclusive scan over (bucket, chunk)
//     emb_scatter_kernel per (table, chunk): SC_W waves x CH/SC_W samples, each wave's
//                        running bucket offsets in LDS, stable ranks inside
//                        a 64-sample step by matching lanes (match_rank)
//   level 2 (tables with sh_t > 0), emb_bucket_sort_kernel: one block per
//     bucket, the same count / scan / stable scatter on id & (2^sh_t - 1).
// Tables with <= 1024 rows (sh_t = 0) are final after level 1.
constexpr int CH = 2048;          // samples per level-1 chunk
constexpr int SC_W = 8;           // emb_scatter_kernel waves per block
constexpr int SC_T = SC_W * WAVE;
constexpr int MAXBK = 4096;       // level-1 buckets per table / level-2 bins
constexpr int SCAN_T = 1024;

struct SortTabs {
  uint32_t base[MAX_TABLES];
  int64_t rows[MAX_TABLES];
  int sh[MAX_TABLES];             // level-1 bucket = id >> sh
  int nbk[MAX_TABLES];            // level-1 buckets
  int nbkb[MAX_TABLES];           // bits of a bucket index (<= 12)
  int gb[MAX_TABLES];             // first global bucket of the table
  int total_bk;                   // hist/offs are [chunk][total_bk] (chunk-major)
};
struct L2Map {                    // level-2 blocks -> (table, bucket)
  int tab[MAX_TABLES];
  int first[MAX_TABLES + 1];
  int n;
};

int nbits64(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

struct SortPlan {
  SortTabs st;
  L2Map l2;
  int total_bk = 0, max_bk = 1, max_low = 1, C = 0;
  bool ok = true;
};

SortPlan make_plan(const int64_t* rows, int nt, int64_t B) {
  SortPlan p;
  memset(&p.st, 0, sizeof(p.st));
  memset(&p.l2, 0, sizeof(p.l2));
  p.C = (int)cdiv(B, CH);
  uint32_t base = 0;
  for (int t = 0; t < nt; ++t) {
    const int nb = nbits64((uint64_t)(rows[t] > 0 ? rows[t] - 1 : 0));
    const int bkb = std::max(10, nb - 12);
    if (bkb > 12) p.ok = false;   // > 2^24 rows
    const int sh = std::max(0, nb - bkb);
    p.st.base[t] = base;
    p.st.rows[t] = rows[t];
    p.st.sh[t] = sh;
    p.st.nbk[t] = (int)(((uint64_t)(rows[t] > 0 ? rows[t] - 1 : 0) >> sh) + 1);
    p.st.nbkb[t] = nbits64((uint64_t)p.st.nbk[t] - 1);
    p.st.gb[t] = p.total_bk;
    p.total_bk += p.st.nbk[t];
    p.max_bk = std::max(p.max_bk, p.st.nbk[t]);
    if (sh > 0) {
      p.l2.tab[p.l2.n] = t;
      p.l2.first[p.l2.n + 1] = p.l2.first[p.l2.n] + p.st.nbk[t];
      ++p.l2.n;
      p.max_low = std::max(p.max_low, 1 << sh);
    }
    base += (uint32_t)rows[t];
  }
  p.st.total_bk = p.total_bk;
  return p;
}

// ids[t*B + b] = clamped id of sample b in table t (the forward gather's
// clamp), table-major for the sort kernels.  A block takes ENT samples: the
// user and item ids one per thread; the block's K categorical columns (one
// contiguous K x ENT int64 run of `cat`) are read coalesced, transposed
// through LDS and written as K coalesced rows.
__global__ __launch_bounds__(ENT) void emb_ids_kernel(SortTabs st, int nt, const int64_t* user,
                                                      const int64_t* item, const int64_t* cat,
                                                      int64_t B, uint32_t* ids) {
  extern __shared__ uint32_t tr[];   // [K][ENT]
  const int K = nt - 2;
  const int64_t b0 = (int64_t)blockIdx.x * ENT;
  const int nb = (int)min<int64_t>(ENT, B - b0);
  auto clampr = [&](int64_t id, int t) {
    const int64_t rows = st.rows[t];
    return (uint32_t)(id < 0 ? 0 : (id >= rows ? rows - 1 : id));
  };
  if (threadIdx.x < nb) {
    const int64_t b = b0 + threadIdx.x;
    ids[b] = clampr(user[b], 0);
    ids[B + b] = clampr(item[b], 1);
  }
  if (K <= 0) return;
  const int64_t* cb = cat + b0 * K;
  for (int j = threadIdx.x; j < nb * K; j += ENT) {
    const int s = j / K, t = j - s * K;
    tr[t * ENT + s] = clampr(cb[j], t + 2);
  }
  __syncthreads();
  if (threadIdx.x < nb)
    for (int t = 0; t < K; ++t) ids[(int64_t)(t + 2) * B + b0 + threadIdx.x] = tr[t * ENT + threadIdx.x];
}

// Lanes holding the same v (v < 2^nb, among `valid` lanes): this lane's rank
// among the lower ones, the group size, and whether it is the group's
// highest lane.  One ballot per value bit (nb <= 12): the peers mask is the
// AND over bits of (bit set ? ballot : ~ballot) -- a fixed cost, unlike a
// loop over the distinct values (up to 64 of them per step here).
__device__ __forceinline__ void match_rank(uint32_t v, bool valid, int nb, int lane, int& rank,
                                           int& cnt, bool& last) {
  uint64_t peers = __ballot(valid);
  for (int i = 0; i < nb; ++i) {
    const bool bit = (v >> i) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  rank = __popcll(peers & below);
  cnt = __popcll(peers);
  last = valid && (peers >> lane) == 1ull;
}

__global__ __launch_bounds__(ENT) void emb_hist_kernel(SortTabs st, const uint32_t* ids,
                                                       int64_t B, int C, uint32_t* hist) {
  extern __shared__ uint32_t h[];
  const int c = blockIdx.x, t = blockIdx.y;
  const int nbk = st.nbk[t], sh = st.sh[t];
  for (int i = threadIdx.x; i < nbk; i += ENT) h[i] = 0u;
  __syncthreads();
  const int64_t b0 = (int64_t)c * CH;
  for (int i = threadIdx.x; i < CH; i += ENT) {
    const int64_t b = b0 + i;
    if (b < B) atomicAdd(&h[ids[(int64_t)t * B + b] >> sh], 1u);
  }
  __syncthreads();
  uint32_t* out = hist + (int64_t)c * st.total_bk + st.gb[t];
  for (int i = threadIdx.x; i < nbk; i += ENT) out[i] = h[i];
}

// hist[chunk][gb_t + bucket] -> t*B + exclusive prefix in (bucket, chunk)
// order.  Thread i owns buckets i, i + SCAN_T, ...: their totals (C
// counts each, loaded 16 at a time), a block scan of the totals, then the
// running offsets along each bucket's chunks.
__global__ __launch_bounds__(SCAN_T) void emb_scan_kernel(SortTabs st, int64_t B, int C,
                                                          uint32_t* hist) {
  constexpr int U = 16;
  __shared__ uint32_t tot[MAXBK];
  __shared__ uint32_t part[SCAN_T];
  const int t = blockIdx.x, tid = threadIdx.x, nbk = st.nbk[t];
  const int64_t TB = st.total_bk;
  uint32_t* seg = hist + st.gb[t];
  for (int bk = tid; bk < nbk; bk += SCAN_T) {
    const uint32_t* row = seg + bk;   // chunk c at row[c * TB]: coalesced across threads
    uint32_t sum = 0;
    for (int c0 = 0; c0 < C; c0 += U) {
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = c0 + u < C ? row[(c0 + u) * TB] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) sum += v[u];
    }
    tot[bk] = sum;
  }
  __syncthreads();
  // exclusive scan of tot[0..nbk): thread-contiguous groups, then across threads
  const int pg = (nbk + SCAN_T - 1) / SCAN_T;
  const int ga = min(nbk, tid * pg), gz = min(nbk, ga + pg);
  uint32_t gsum = 0;
  for (int i = ga; i < gz; ++i) gsum += tot[i];
  part[tid] = gsum;
  __syncthreads();
  for (int o = 1; o < SCAN_T; o <<= 1) {
    const uint32_t v = tid >= o ? part[tid - o] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - gsum;
  for (int i = ga; i < gz; ++i) {
    const uint32_t v = tot[i];
    tot[i] = run;
    run += v;
  }
  __syncthreads();
  for (int bk = tid; bk < nbk; bk += SCAN_T) {
    uint32_t* row = seg + bk;
    uint32_t r = (uint32_t)((int64_t)t * B) + tot[bk];
    for (int c0 = 0; c0 < C; c0 += U) {
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = c0 + u < C ? row[(c0 + u) * TB] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (c0 + u < C) {
          row[(c0 + u) * TB] = r;
          r += v[u];
        }
    }
  }
}

__global__ __launch_bounds__(SC_T) void emb_scatter_kernel(SortTabs st, int nt, const uint32_t* ids,
                                                          int64_t B, int C, const uint32_t* offs,
                                                          uint32_t* mid_k, uint32_t* mid_v,
                                                          uint32_t* fin_k, uint32_t* fin_v) {
  extern __shared__ uint32_t wh[];   // [SC_W][nbk]: per-wave counts, then running offsets
  // XCD-aware block map: every chunk of table t runs on XCD t % 8, so the
  // scattered 4-B stores into the table's output range combine in one L2
  const int L8 = blockIdx.x & 7, k8 = blockIdx.x >> 3, jt = k8 / C;
  const int c = k8 - jt * C, t = L8 + 8 * jt;
  if (t >= nt) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nbk = st.nbk[t], sh = st.sh[t];
  for (int i = threadIdx.x; i < SC_W * nbk; i += SC_T) wh[i] = 0u;
  __syncthreads();
  const int64_t b0 = (int64_t)c * CH + (int64_t)w * (CH / SC_W);
  constexpr int Q = CH / SC_W / WAVE;
  uint32_t id[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int64_t b = b0 + q * WAVE + lane;
    id[q] = b < B ? ids[(int64_t)t * B + b] : 0u;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (b0 + q * WAVE + lane < B) atomicAdd(&wh[w * nbk + (id[q] >> sh)], 1u);
  __syncthreads();
  {
    constexpr int J = MAXBK / SC_T;
    const uint32_t* orow = offs + (int64_t)c * st.total_bk + st.gb[t];
    uint32_t ov[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int i = threadIdx.x + j * SC_T;
      ov[j] = i < nbk ? orow[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int i = threadIdx.x + j * SC_T;
      if (i < nbk) {
        uint32_t acc = ov[j];
        for (int ww = 0; ww < SC_W; ++ww) {
          const uint32_t v = wh[ww * nbk + i];
          wh[ww * nbk + i] = acc;
          acc += v;
        }
      }
    }
  }
  __syncthreads();
  uint32_t* ok_ = sh ? mid_k : fin_k;
  uint32_t* ov_ = sh ? mid_v : fin_v;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int64_t b = b0 + q * WAVE + lane;
    const bool valid = b < B;
    const uint32_t bk = id[q] >> sh;
    int rank, cnt;
    bool last;
    match_rank(bk, valid, st.nbkb[t], lane, rank, cnt, last);
    uint32_t* slot = &wh[w * nbk + (valid ? bk : 0)];
    const uint32_t pos = *slot + rank;
    if (valid) {
      ok_[pos] = st.base[t] + id[q];
      ov_[pos] = (uint32_t)b;
    }
    if (last) *slot = pos - rank + cnt;
  }
}

__global__ __launch_bounds__(ENT) void emb_bucket_sort_kernel(SortTabs st, L2Map mp, int64_t B,
                                                              int C, const uint32_t* offs,
                                                              const uint32_t* mid_k,
                                                              const uint32_t* mid_v,
                                                              uint32_t* fin_k, uint32_t* fin_v) {
  extern __shared__ uint32_t wh[];   // [4][nlow]
  __shared__ uint32_t part[ENT];
  int j = 0;
  while (j + 1 < mp.n && (int)blockIdx.x >= mp.first[j + 1]) ++j;
  const int t = mp.tab[j], bk = (int)blockIdx.x - mp.first[j];
  const int sh = st.sh[t], nlow = 1 << sh, nbk = st.nbk[t];
  const uint32_t mask = (uint32_t)nlow - 1u, base = st.base[t];
  const int64_t start = offs[st.gb[t] + bk];   // chunk 0 row of offs
  const int64_t end = bk + 1 < nbk ? (int64_t)offs[st.gb[t] + bk + 1]
                                   : (int64_t)(t + 1) * B;
  const int64_t ne = end - start;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (ne <= 1) {
    if (ne == 1 && tid == 0) { fin_k[start] = mid_k[start]; fin_v[start] = mid_v[start]; }
    return;
  }
  const int64_t per = (ne + 3) / 4;
  const int64_t a = min(end, start + w * per), z = min(end, a + per);
  for (int i = tid; i < 4 * nlow; i += ENT) wh[i] = 0u;
  __syncthreads();
  for (int64_t p = a + lane; p < z; p += WAVE) atomicAdd(&wh[w * nlow + ((mid_k[p] - base) & mask)], 1u);
  __syncthreads();
  // exclusive scan over (low bin, wave): each thread a contiguous range of bins
  const int pl = (nlow + ENT - 1) / ENT;
  const int la = min(nlow, tid * pl), lz = min(nlow, la + pl);
  uint32_t sum = 0;
  for (int l = la; l < lz; ++l)
    for (int ww = 0; ww < 4; ++ww) sum += wh[ww * nlow + l];
  part[tid] = sum;
  __syncthreads();
  for (int o = 1; o < ENT; o <<= 1) {
    const uint32_t v = tid >= o ? part[tid - o] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - sum;
  for (int l = la; l < lz; ++l)
    for (int ww = 0; ww < 4; ++ww) {
      const uint32_t v = wh[ww * nlow + l];
      wh[ww * nlow + l] = run;
      run += v;
    }
  __syncthreads();
  // stable scatter, 64 entries per step, the next step's loads in flight
  int64_t p = a + lane;
  uint32_t kn = p < z ? mid_k[p] : 0u, vn = p < z ? mid_v[p] : 0u;
  for (int64_t p0 = a; p0 < z; p0 += WAVE) {
    const bool valid = p0 + lane < z;
    const uint32_t key = kn, v = vn;
    p = p0 + WAVE + lane;
    if (p0 + WAVE < z) { kn = p < z ? mid_k[p] : 0u; vn = p < z ? mid_v[p] : 0u; }
    const uint32_t low = (key - base) & mask;
    int rank, cnt;
    bool last;
    match_rank(low, valid, sh, lane, rank, cnt, last);
    uint32_t* slot = &wh[w * nlow + (valid ? low : 0)];
    const uint32_t pos = *slot + rank;
    if (valid) {
      fin_k[start + pos] = key;
      fin_v[start + pos] = v;
    }
    if (last) *slot = pos - rank + cnt;
  }
}

// Tables of more than 2^24 rows (beyond the two counting levels): one stable
// LSD radix sort (rocPRIM) of key = base_t + id, value = sample over all
// tables at once.  Every table contributes exactly B keys and the keys of
// table t lie in [base_t, base_t + rows_t), so table t still lands in
// [t*B, (t+1)*B) in ascending (id, sample) order: the same output as the
// counting sort, at the cost of ~4 8-bit passes.
__global__ __launch_bounds__(ENT) void emb_keys_kernel(SortTabs st, const uint32_t* ids, int64_t B,
                                                       int64_t n, uint32_t* keys, uint32_t* vals) {
  const int64_t i = (int64_t)blockIdx.x * ENT + threadIdx.x;
  if (i >= n) return;
  const int t = (int)(i / B);
  keys[i] = st.base[t] + ids[i];
  vals[i] = (uint32_t)(i - (int64_t)t * B);
}

size_t radix_tmp_bytes(int64_t n, int end_bit) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n, 0u,
                                  (unsigned)end_bit, (hipStream_t)0);
  return bytes;
}

uint64_t total_rows(const int64_t* rows, int nt) {
  uint64_t total = 0;
  for (int i = 0; i < nt; ++i) total += (uint64_t)rows[i];
  return total;
}

template <int VEC> struct Vec;
template <> struct Vec<1> {
  typedef float T;
  // a + c * v rounded twice (never contracted to an fma: the test restates it)
  static __device__ __forceinline__ T axpy(T a, float c, T v) {
#pragma clang fp contract(off)
    const T m = c * v;
    return a + m;
  }
  static __device__ __forceinline__ T ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, T v) { *p = v; }
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T shfl(T v, int src) { return __shfl(v, src); }
};
template <> struct Vec<4> {
  typedef f32x4 T;
  static __device__ __forceinline__ T axpy(T a, float c, T v) {
#pragma clang fp contract(off)
    const T m = c * v;
    return a + m;
  }
  static __device__ __forceinline__ T ld(const float* p) { return *reinterpret_cast<const T*>(p); }
  static __device__ __forceinline__ void st(float* p, T v) { *reinterpret_cast<T*>(p) = v; }
  static __device__ __forceinline__ T zero() { return T{0.f, 0.f, 0.f, 0.f}; }
  static __device__ __forceinline__ T shfl(T v, int src) {
    return T{__shfl(v[0], src), __shfl(v[1], src), __shfl(v[2], src), __shfl(v[3], src)};
  }
};

template <int NV>
__device__ void emb_huge_final(const EmbTabs& et, int64_t B, int64_t n, int64_t g,
                               const float* hp, int hps, int accumulate, int lane);

// One thread per sorted position; the head of a run of <= LIM entries sums
// it in ascending sample order: the deep dx0 segments and the NV cross
// coefficients, then row = deep + sum_k csum_k V_k.  Latency, not bandwidth,
// bounds this kernel (a few KB per wave, scattered rows), so no load waits
// on another it does not depend on: the run's keys and samples are loaded
// together, and its dx0 rows EG entries at a time (UNR column groups of VEC
// per pass).
template <int VEC, int NV>
__global__ __launch_bounds__(ENT) void emb_runs_short_kernel(EmbTabs et, int nt, int64_t B,
                                                             const uint32_t* ks,
                                                             const uint32_t* vs,
                                                             const float* dx0, int ld,
                                                             const float* coef,
                                                             const float* hp, int hps,
                                                             int64_t nseg, int accumulate) {
  typedef Vec<VEC> V;
  typedef typename V::T T;
  constexpr int UNR = 16 / VEC;   // 16 columns per pass
  constexpr int EG = 2;           // entries whose loads are in flight together
  const int64_t i = (int64_t)blockIdx.x * ENT + threadIdx.x;
  const int64_t n = (int64_t)nt * B, nbh = (n + ENT - 1) / ENT;   // head-position blocks
  if ((int64_t)blockIdx.x >= nbh) {   // huge-run finalisation waves
    const int64_t g = ((int64_t)blockIdx.x - nbh) * (ENT / WAVE) + (threadIdx.x >> 6);
    if (g < nseg) emb_huge_final<NV>(et, B, n, g, hp, hps, accumulate, threadIdx.x & 63);
    return;
  }
  if (i >= n) return;
  const int t = (int)(i / B);
  const int64_t t0 = (int64_t)t * B, t1 = t0 + B;
  const uint32_t k = ks[i];
  if (i > t0 && ks[i - 1] == k) return;   // not the head of its run
  if (et.touched) et.touched[k] = 1;      // every run (short, long, huge) has its head here
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
  // cross coefficients, summed in entry order
  float csum[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) csum[v] = 0.f;
#pragma unroll
  for (int q0 = 0; q0 < LIM; q0 += EG) {
    if (q0 >= len) break;
    float cf[EG][NV];
#pragma unroll
    for (int q = 0; q < EG; ++q)
#pragma unroll
      for (int v = 0; v < NV; ++v) cf[q][v] = q0 + q < len ? coef[(int64_t)smp[q0 + q] * NV + v] : 0.f;
#pragma unroll
    for (int q = 0; q < EG; ++q)
      if (q0 + q < len)
#pragma unroll
        for (int v = 0; v < NV; ++v) csum[v] += cf[q][v];
  }
  const int w = et.width[t];
  const float* src = dx0 + et.off[t];
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
        const float* row = src + (int64_t)smp[q0 + q] * ld + c;
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
        const int col = et.off[t] + c + u * VEC;
        T r = acc[u];
#pragma unroll
        for (int v = 0; v < NV; ++v) r = V::axpy(r, csum[v], V::ld(et.V[v] + col));
        float* p = dst + c + u * VEC;
        V::st(p, accumulate ? V::ld(p) + r : r);
      }
  }
}

// Sums over the entries [lo, hi) of run k (table t), walked WAVE entries at
// a time from lo: lane L holds entry p+L's key and sample (coalesced loads,
// the next block's issued before this block's dx0 rows), the column groups
// of VEC (column block cb) sit across lanes and the block's entries across
// the remaining S = 64/Gb lane slots (slot s takes entries s, s+S, ... of
// every block, summing their deep segments and cross coefficients in
// ascending order), slots added in ascending order.  Returns, in the slot-0
// lanes, the deep sum of their columns (tot) and in every lane the NV
// coefficient sums (ctot).  SPLIT (Gb >= NV): lane (slot, cg < NV) sums
// coefficient cg of its slot's entries instead of every lane summing all NV.
template <int VEC, int NV, bool SPLIT>
__device__ __forceinline__ void piece_sums(const EmbTabs& et, int t, uint32_t k, int64_t lo,
                                           int64_t hi, const uint32_t* ks, const uint32_t* vs,
                                           const float* dx0, int ld, const float* coef, int cb,
                                           int lane, typename Vec<VEC>::T& tot,
                                           float (&ctot)[NV]) {
  typedef Vec<VEC> V;
  typedef typename V::T T;
  constexpr int QMAX = 8;   // entries per slot per block held in flight (S >= 8)
  const int G = et.width[t] / VEC;
  const float* src = dx0 + et.off[t];
  const int Gb = G - cb < WAVE ? G - cb : WAVE;
  const int S = WAVE / Gb, slot = lane / Gb, cg = lane - slot * Gb;
  const int col = (cb + cg) * VEC;
  const bool act = slot < S;
  T acc = V::zero();
  float csum[SPLIT ? 1 : NV];
#pragma unroll
  for (int v = 0; v < (SPLIT ? 1 : NV); ++v) csum[v] = 0.f;
  int64_t p = lo;
  uint32_t kn = p + lane < hi ? ks[p + lane] : ~0u;
  uint32_t sn = p + lane < hi ? vs[p + lane] : 0u;
  for (;;) {
    const int nb = __popcll(__ballot(kn == k));   // the piece's entries in this block: a prefix
    const int smp = (int)sn;
    const int64_t pn = p + WAVE;
    if (nb == WAVE) {   // the piece may go on: fetch the next block now
      kn = pn + lane < hi ? ks[pn + lane] : ~0u;
      sn = pn + lane < hi ? vs[pn + lane] : 0u;
    }
    for (int q0 = 0; S * q0 < WAVE; q0 += QMAX) {   // uniform trip count
      T x[QMAX];
      float cf[QMAX][SPLIT ? 1 : NV];
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        const int j = slot + S * (q0 + q);
        const int b = __shfl(smp, j & 63);
        const bool ok = act && j < nb;
        x[q] = ok ? V::ld(src + (int64_t)b * ld + col) : V::zero();
        if constexpr (SPLIT)
          cf[q][0] = ok && cg < NV ? coef[(int64_t)b * NV + cg] : 0.f;
        else
#pragma unroll
          for (int v = 0; v < NV; ++v) cf[q][v] = ok ? coef[(int64_t)b * NV + v] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < QMAX; ++q)
        if (act && slot + S * (q0 + q) < nb) {
          acc += x[q];
#pragma unroll
          for (int v = 0; v < (SPLIT ? 1 : NV); ++v) csum[v] += cf[q][v];
        }
    }
    if (nb < WAVE) break;
    p = pn;
  }
  tot = acc;
  constexpr int NC = SPLIT ? 1 : NV;
#pragma unroll
  for (int v = 0; v < NC; ++v) ctot[v] = csum[v];
  for (int s = 1; s < S; ++s) {   // wave-uniform trip count
    const int src_l = (s * Gb + cg) & 63;
    const T o = V::shfl(acc, src_l);
    float oc[NC];
#pragma unroll
    for (int v = 0; v < NC; ++v) oc[v] = __shfl(csum[v], src_l);
    if (slot == 0) {
      tot += o;
#pragma unroll
      for (int v = 0; v < NC; ++v) ctot[v] += oc[v];
    }
  }
  if constexpr (SPLIT) {   // coefficient v's total sits in lane v (slot 0, cg v)
    const float mine = ctot[0];
#pragma unroll
    for (int v = 0; v < NV; ++v) ctot[v] = __shfl(mine, v);
  } else {
#pragma unroll
    for (int v = 0; v < NV; ++v) ctot[v] = __shfl(ctot[v], 0);
  }
}

// Huge runs (> HSEG entries, e.g. one id taking a large share of the batch)
// are cut at the global HSEG-position segment boundaries: the wave of segment
// g writes the partial sums of the (at most two) huge-run pieces inside it
// to hp[g][slot] = {key, run start, run end, NV coefficient sums, w deep
// sums}; the wave of the segment where a huge run starts adds its pieces in
// segment order (emb_huge_final, run by the short kernel's extra waves).
constexpr int HSEG = 2048;

__device__ __forceinline__ int64_t lower_key(const uint32_t* ks, int64_t lo, int64_t hi, uint32_t k) {
  while (lo < hi) {   // first position in [lo, hi) with key >= k
    const int64_t mid = (lo + hi) >> 1;
    if (ks[mid] < k) lo = mid + 1; else hi = mid;
  }
  return lo;
}

template <int VEC, int NV, bool SPLIT>
__device__ void emb_huge_partial(const EmbTabs& et, int64_t B, int64_t n, int64_t g,
                                 const uint32_t* ks, const uint32_t* vs, const float* dx0,
                                 int ld, const float* coef, float* hp, int hps, int lane) {
  typedef typename Vec<VEC>::T T;
  const int64_t s0 = g * HSEG, s1 = min(n, s0 + HSEG);
  for (int slot = 0; slot < 2; ++slot) {
    float* out = hp + (g * 2 + slot) * (int64_t)hps;
    uint32_t* hdr = reinterpret_cast<uint32_t*>(out);
    const int64_t p = slot == 0 ? s0 : s1 - 1;
    const uint32_t k = ks[p];
    const int t = (int)(p / B);
    const int64_t t0 = (int64_t)t * B, t1 = t0 + B;
    bool cand = !(slot == 1 && k == ks[s0]);   // the same run as slot 0
    // a run longer than HSEG through p reaches p - HSEG/2 or p + HSEG/2
    if (cand) {
      const bool l = p - HSEG / 2 >= t0 && ks[p - HSEG / 2] == k;
      const bool r = p + HSEG / 2 < t1 && ks[p + HSEG / 2] == k;
      cand = l || r;
    }
    int64_t rs = 0, re = 0;
    if (cand) {
      rs = lower_key(ks, t0, p, k);
      re = lower_key(ks, p + 1, t1, k + 1);
      cand = re - rs > HSEG;
    }
    if (!cand) {
      if (lane == 0) hdr[0] = ~0u;
      continue;
    }
    const int64_t lo = max(rs, s0), hi = min(re, s1);
    const int G = et.width[t] / VEC;
    for (int cb = 0; cb < G; cb += WAVE) {
      T tot;
      float ctot[NV];
      piece_sums<VEC, NV, SPLIT>(et, t, k, lo, hi, ks, vs, dx0, ld, coef, cb, lane, tot, ctot);
      const int Gb = G - cb < WAVE ? G - cb : WAVE;
      if (lane < Gb) Vec<VEC>::st(out + 3 + 8 + (cb + lane) * VEC, tot);
      if (cb == 0 && lane < NV) out[3 + lane] = ctot[lane];
    }
    if (lane == 0) { hdr[0] = k; hdr[1] = (uint32_t)rs; hdr[2] = (uint32_t)re; }
  }
}

// the wave of segment g finalises every huge run that starts inside it
template <int NV>
__device__ void emb_huge_final(const EmbTabs& et, int64_t B, int64_t n, int64_t g,
                               const float* hp, int hps, int accumulate, int lane) {
  for (int slot = 0; slot < 2; ++slot) {
    const float* in = hp + (g * 2 + slot) * (int64_t)hps;
    const uint32_t* hdr = reinterpret_cast<const uint32_t*>(in);
    const uint32_t k = hdr[0];
    if (k == ~0u) continue;
    const int64_t rs = hdr[1], re = hdr[2];
    if (rs < g * HSEG) continue;   // starts in an earlier segment
    const int t = (int)(rs / B);
    const int w = et.width[t];
    const int64_t g1 = (re - 1) / HSEG;
    float* dst = et.grad[t] + (int64_t)(k - et.base[t]) * w;
    float csum = 0.f;   // lane v < NV: coefficient v
    for (int c0 = 0; c0 < w; c0 += WAVE) {
      const int c = c0 + lane;
      float acc = 0.f;
      for (int64_t gg = g; gg <= g1; ++gg) {   // pieces in segment order
        const float* pc = hp + (gg * 2) * (int64_t)hps;
        if (reinterpret_cast<const uint32_t*>(pc)[0] != k) pc += hps;   // its slot 1
        if (c < w) acc += pc[3 + 8 + c];
        if (c0 == 0 && lane < NV) csum += pc[3 + lane];
      }
      float cs[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) cs[v] = __shfl(csum, v);
      if (c < w) {
        float r = acc;
#pragma unroll
        for (int v = 0; v < NV; ++v) r = Vec<1>::axpy(r, cs[v], et.V[v][et.off[t] + c]);
        dst[c] = accumulate ? dst[c] + r : r;
      }
    }
  }
}

// One wave per long run (LIM < length <= HSEG); the wave owning the run's
// head position (64 positions per wave) reduces it with piece_sums and writes
// row = deep + sum_k csum_k V_k.  Blocks past the head-position range are the
// huge-run partial waves (one per HSEG segment).
template <int VEC, int NV, bool SPLIT>
__global__ __launch_bounds__(ENT) void emb_runs_long_kernel(EmbTabs et, int64_t B, int64_t n,
                                                            const uint32_t* ks,
                                                            const uint32_t* vs,
                                                            const float* dx0, int ld,
                                                            const float* coef, float* hp,
                                                            int hps, int64_t nseg,
                                                            int accumulate) {
  typedef Vec<VEC> V;
  typedef typename V::T T;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (ENT / WAVE) + (threadIdx.x >> 6);
  const int64_t nwh = (n + WAVE - 1) / WAVE;   // head-position waves
  if (wave >= nwh) {
    if (wave - nwh < nseg)
      emb_huge_partial<VEC, NV, SPLIT>(et, B, n, wave - nwh, ks, vs, dx0, ld, coef, hp, hps, lane);
    return;
  }
  // this wave's 64 positions: which start a run longer than LIM (not huge)
  const int64_t base = wave * WAVE;
  bool head = false;
  {
    const int64_t i = base + lane;
    if (i < n) {
      const int t = (int)(i / B);
      const int64_t t0 = (int64_t)t * B, t1 = t0 + B;
      const uint32_t k = ks[i];
      head = (i == t0 || ks[i - 1] != k) && i + LIM < t1 && ks[i + LIM] == k &&
             !(i + HSEG < t1 && ks[i + HSEG] == k);
    }
  }
  for (uint64_t hm = __ballot(head); hm; hm &= hm - 1) {
    const int64_t i = base + __builtin_ctzll(hm);
    const uint32_t k = ks[i];
    const int t = (int)(i / B);
    const int64_t t1 = (int64_t)(t + 1) * B;
    const int w = et.width[t], G = w / VEC;
    float* dst = et.grad[t] + (int64_t)(k - et.base[t]) * w;
    for (int cb = 0; cb < G; cb += WAVE) {
      T tot;
      float ctot[NV];
      piece_sums<VEC, NV, SPLIT>(et, t, k, i, t1, ks, vs, dx0, ld, coef, cb, lane, tot, ctot);
      const int Gb = G - cb < WAVE ? G - cb : WAVE;
      if (lane < Gb) {   // slot-0 lanes
        const int col = (cb + lane) * VEC;
        const int xc = et.off[t] + col;
        T r = tot;
#pragma unroll
        for (int v = 0; v < NV; ++v) r = V::axpy(r, ctot[v], V::ld(et.V[v] + xc));
        float* q = dst + col;
        V::st(q, accumulate ? V::ld(q) + r : r);
      }
    }
  }
}

bool vec4_ok(const EmbBwdDesc& e, const float* dx0, int ld) {
  if (((uintptr_t)dx0 & 15) || ld % 4) return false;
  for (int t = 0; t < e.n_tab; ++t)
    if (e.width[t] % 4 || e.off[t] % 4 || ((uintptr_t)e.grad[t] & 15)) return false;
  for (int k = 0; k < e.nv; ++k)
    if ((uintptr_t)e.V[k] & 15) return false;
  return true;
}

}  // namespace

namespace {
// huge-run piece slots: {key, run start, run end, 8 coefficients, widest row}
int huge_stride(const int* width, int nt) {
  int w = 0;
  for (int t = 0; t < nt; ++t) w = std::max(w, width[t]);
  return (3 + 8 + w + 3) & ~3;
}
int64_t huge_segs(int nt, int64_t B) { return cdiv((int64_t)nt * B, (int64_t)HSEG); }
}  // namespace

size_t emb_sort_tmp_bytes(const int64_t* rows, const int* width, int nt, int64_t B) {
  const SortPlan p = make_plan(rows, nt, B);
  // the sort's counts (or the radix sort's scratch) are dead once the sort
  // is done: the sums reuse them for the huge-run pieces
  const size_t pieces = (size_t)huge_segs(nt, B) * 2 * huge_stride(width, nt) * 4;
  if (!p.ok) {
    const uint64_t total = total_rows(rows, nt);
    return std::max(radix_tmp_bytes((int64_t)nt * B, std::max(1, nbits64(total - 1))), pieces);
  }
  return std::max((size_t)p.total_bk * (size_t)std::max(p.C, 1) * 4, pieces);
}

dcnr_status emb_sort(const EmbBwdDesc& e, const int64_t* user, const int64_t* item,
                     const int64_t* cat, int64_t B, const EmbSortBufs& sb, hipStream_t s) {
  const int64_t n = (int64_t)e.n_tab * B;
  if (n <= 0) return DCNR_OK;
  const uint64_t total = total_rows(e.rows, e.n_tab);
  const SortPlan p = make_plan(e.rows, e.n_tab, B);
  if (total >= (1ull << 32) || n >= (1ll << 32)) {   // 32-bit sort keys / positions
    set_error("embedding backward: %llu table rows in all or %lld ids (>= 2^32) unsupported",
              (unsigned long long)total, (long long)n);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (!p.ok) {   // a table of > 2^24 rows: one stable radix sort (emb_keys_kernel)
    const int end_bit = std::max(1, nbits64(total - 1));
    size_t need = radix_tmp_bytes(n, end_bit);
    if (need > sb.tmp_bytes) {
      set_error("embedding backward: radix-sort scratch too small");
      return DCNR_WORKSPACE_TOO_SMALL;
    }
    hipLaunchKernelGGL(emb_ids_kernel, dim3((unsigned)cdiv(B, ENT)), dim3(ENT),
                       (size_t)std::max(e.n_tab - 2, 1) * ENT * 4, s, p.st, e.n_tab, user, item,
                       cat, B, sb.ids);
    DCNR_LAUNCH_CHECK();
    hipLaunchKernelGGL(emb_keys_kernel, dim3((unsigned)cdiv(n, ENT)), dim3(ENT), 0, s, p.st, sb.ids,
                       B, n, sb.keys, sb.vals);
    DCNR_LAUNCH_CHECK();
    size_t tb = sb.tmp_bytes;
    DCNR_HIP(rocprim::radix_sort_pairs(sb.tmp, tb, (const uint32_t*)sb.keys, sb.keys_s,
                                       (const uint32_t*)sb.vals, sb.vals_s, (size_t)n, 0u,
                                       (unsigned)end_bit, s));
    return DCNR_OK;
  }
  if ((size_t)p.total_bk * p.C * 4 > sb.tmp_bytes) {
    set_error("embedding backward: sort scratch too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  uint32_t* hist = (uint32_t*)sb.tmp;
  // dynamic LDS above the 64 KiB default
  const size_t lds_bk = (size_t)SC_W * p.max_bk * 4, lds_low = (size_t)4 * p.max_low * 4;
  if (lds_bk > 65536) TRY_ST(set_max_dyn_lds((const void*)emb_scatter_kernel, lds_bk));
  if (lds_low + ENT * 4 > 65536) TRY_ST(set_max_dyn_lds((const void*)emb_bucket_sort_kernel, lds_low));
  const dim3 gc((unsigned)p.C, (unsigned)e.n_tab);
  hipLaunchKernelGGL(emb_ids_kernel, dim3((unsigned)cdiv(B, ENT)), dim3(ENT),
                     (size_t)std::max(e.n_tab - 2, 1) * ENT * 4, s, p.st, e.n_tab, user, item,
                     cat, B, sb.ids);
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(emb_hist_kernel, gc, dim3(ENT), (size_t)p.max_bk * 4, s, p.st, sb.ids, B,
                     p.C, hist);
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(emb_scan_kernel, dim3((unsigned)e.n_tab), dim3(SCAN_T), 0, s, p.st, B, p.C,
                     hist);
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(emb_scatter_kernel, dim3((unsigned)(8 * cdiv(e.n_tab, 8) * p.C)), dim3(SC_T),
                     lds_bk, s, p.st, e.n_tab, sb.ids, B, p.C, hist, sb.keys, sb.vals,
                     sb.keys_s, sb.vals_s);
  DCNR_LAUNCH_CHECK();
  if (p.l2.n > 0) {
    hipLaunchKernelGGL(emb_bucket_sort_kernel, dim3((unsigned)p.l2.first[p.l2.n]), dim3(ENT),
                       lds_low, s, p.st, p.l2, B, p.C, hist, sb.keys, sb.vals, sb.keys_s,
                       sb.vals_s);
    DCNR_LAUNCH_CHECK();
  }
  return DCNR_OK;
}

namespace {

// ------------------------------------------------------- touched rows
// One block per asked table walks its B sorted keys in chunks of TR_T * TR_U
// positions: a position is a run head when its key differs from the previous
// one; heads are compacted in order by a block scan (ascending rows, as the
// sort left them) and counted per owner in LDS.  ~2 x 512 KB per table: a
// latency-bound single-CU stream, off the backward's critical path.
constexpr int TR_T = 1024, TR_U = 4, TR_MAXW = 64;

__global__ __launch_bounds__(TR_T) void emb_touched_kernel(TouchedArgs a, const uint32_t* keys,
                                                           int64_t B, int64_t* out,
                                                           int64_t* table_counts,
                                                           int64_t* owner_counts) {
  __shared__ uint32_t wsum[TR_T / WAVE];
  __shared__ int own[TR_MAXW];
  const int i = blockIdx.x, t = a.tab[i], tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int r = tid; r < TR_MAXW; r += TR_T) own[r] = 0;
  __syncthreads();
  const uint32_t* k = keys + (int64_t)t * B;
  int64_t* o = out + (int64_t)i * B;
  const uint32_t base = a.base[i];
  const int64_t eoff = a.elem_off[i], wd = a.width[i];
  int64_t total = 0;
  for (int64_t c0 = 0; c0 < B; c0 += (int64_t)TR_T * TR_U) {
    uint32_t kv[TR_U];
    bool head[TR_U];
    uint32_t cnt = 0;
#pragma unroll
    for (int u = 0; u < TR_U; ++u) {   // thread-contiguous positions: in-order compaction
      const int64_t p = c0 + (int64_t)tid * TR_U + u;
      kv[u] = p < B ? k[p] : 0u;
      head[u] = p < B && (p == 0 || k[p - 1] != kv[u]);
      cnt += head[u];
    }
    // block exclusive scan of the per-thread head counts
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    if (lane == WAVE - 1) wsum[w] = incl;
    __syncthreads();
    uint32_t wpre = 0, all = 0;
    for (int j = 0; j < TR_T / WAVE; ++j) {
      const uint32_t v = wsum[j];
      wpre += j < w ? v : 0u;
      all += v;
    }
    uint32_t pos = wpre + incl - cnt;
#pragma unroll
    for (int u = 0; u < TR_U; ++u)
      if (head[u]) {
        const int64_t off = eoff + (int64_t)(kv[u] - base) * wd;
        o[total + pos++] = off;
        const int64_t r = off / a.shard;
        if (r < a.world) atomicAdd(&own[r], 1);
      }
    total += all;
    __syncthreads();   // wsum reused
  }
  __syncthreads();
  if (tid == 0) table_counts[i] = total;
  for (int r = tid; r < a.world; r += TR_T)
    if (own[r]) atomicAdd((unsigned long long*)&owner_counts[r], (unsigned long long)own[r]);
}

}  // namespace

dcnr_status emb_touched_rows(const TouchedArgs& a, const EmbSortBufs& sb, int64_t B, int64_t* out,
                             int64_t* table_counts, int64_t* owner_counts, hipStream_t s) {
  if (a.n < 1 || a.world < 1 || a.world > TR_MAXW || a.shard < 1) {
    set_error("emb_touched_rows: %d tables, world %d (1..%d), shard %lld", a.n, a.world, TR_MAXW,
              (long long)a.shard);
    return DCNR_BAD_ARG;
  }
  DCNR_HIP(hipMemsetAsync(owner_counts, 0, (size_t)a.world * 8, s));
  if (B <= 0) {
    DCNR_HIP(hipMemsetAsync(table_counts, 0, (size_t)a.n * 8, s));
    return DCNR_OK;
  }
  hipLaunchKernelGGL(emb_touched_kernel, dim3((unsigned)a.n), dim3(TR_T), 0, s, a, sb.keys_s, B, out,
                     table_counts, owner_counts);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

namespace {

// ------------------------------------------------ sparse exchange (DP)
// Pack: table t's touched rows (offsets offs[t][0 .. tcnt[t]), ascending)
// go to positions [sum_{u<t} tcnt[u], ...) of the send buffers -- the
// tables in flat order, so the whole list is ascending and grouped by owner.
// One thread per 16 B of a row (width % 4 == 0) or per float.
template <int V>
__global__ __launch_bounds__(256) void sparse_pack_kernel(const float* __restrict__ grad,
                                                          const int64_t* __restrict__ offs, int64_t ld,
                                                          const int64_t* __restrict__ tcnt, int width,
                                                          int64_t* __restrict__ out_off,
                                                          float* __restrict__ out_rows) {
  const int t = blockIdx.y;
  int64_t base = 0;
  for (int u = 0; u < t; ++u) base += tcnt[u];
  const int64_t n = tcnt[t];
  const int per = width / V;   // threads per row
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * per;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / per;
    const int c = (int)(e % per) * V;
    const int64_t o = offs[(int64_t)t * ld + i];
    if (c == 0) out_off[base + i] = o;
    if constexpr (V == 4) {
      float* d = out_rows + (base + i) * width + c;
      if ((o & 3) == 0) {
        *reinterpret_cast<float4*>(d) = *reinterpret_cast<const float4*>(grad + o + c);
      } else {   // a caller's offset off the 16-B grid (FusedTrainer's never are)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = grad[o + c + j];
      }
    } else {
      out_rows[(base + i) * width + c] = grad[o + c];
    }
  }
}

// Accumulate one source's rows (distinct offsets) into the shard [lo, lo +
// elems): a plain read-add-write, since no two of them share a row; the
// sources are launched in rank order, so every shard row is summed
// 0 + g_0 + g_1 + ... whatever the scheduling.  Offsets outside the shard
// (none, from sparse_pack's owner grouping) are skipped.
template <int V>
__global__ __launch_bounds__(256) void sparse_add_kernel(float* __restrict__ shard, int64_t lo, int64_t elems,
                                                         int width, const int64_t* __restrict__ offs,
                                                         const float* __restrict__ rows, int64_t n) {
  const int per = width / V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * per;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / per;
    const int c = (int)(e % per) * V;
    const int64_t r = offs[i] - lo;
    if (r < 0 || r + width > elems) continue;
    if constexpr (V == 4) {
      if (r & 3) {   // a row off the 16-B grid: scalar adds
#pragma unroll
        for (int j = 0; j < 4; ++j) shard[r + c + j] += rows[i * width + c + j];
        continue;
      }
      float4* d = reinterpret_cast<float4*>(shard + r + c);
      const float4 g = *reinterpret_cast<const float4*>(rows + i * width + c);
      float4 v = *d;
      v.x += g.x; v.y += g.y; v.z += g.z; v.w += g.w;
      *d = v;
    } else {
      shard[r + c] += rows[i * width + c];
    }
  }
}

}  // namespace

dcnr_status sparse_pack(const float* grad, const int64_t* offs, int64_t ld, const int64_t* tcnt, int n_tables,
                        int width, int64_t* out_off, float* out_rows, hipStream_t s) {
  if (ld <= 0 || n_tables < 1) return DCNR_OK;
  const bool v4 = width % 4 == 0 && (uintptr_t)grad % 16 == 0 && (uintptr_t)out_rows % 16 == 0;
  const int per = v4 ? width / 4 : width;
  const unsigned bx = (unsigned)std::min<int64_t>(cdiv(ld * per, 256), 2048);
  if (v4)
    hipLaunchKernelGGL(sparse_pack_kernel<4>, dim3(bx, n_tables), dim3(256), 0, s, grad, offs, ld, tcnt, width,
                       out_off, out_rows);
  else
    hipLaunchKernelGGL(sparse_pack_kernel<1>, dim3(bx, n_tables), dim3(256), 0, s, grad, offs, ld, tcnt, width,
                       out_off, out_rows);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status sparse_accumulate(float* shard, int64_t lo, int64_t elems, int width, const int64_t* offs,
                              const float* rows, const int64_t* counts, int n_sources, hipStream_t s) {
  DCNR_HIP(hipMemsetAsync(shard, 0, (size_t)elems * 4, s));
  const bool v4 = width % 4 == 0 && lo % 4 == 0 && (uintptr_t)shard % 16 == 0 && (uintptr_t)rows % 16 == 0;
  int64_t pos = 0;
  for (int r = 0; r < n_sources; ++r) {   // rank order: one launch per source
    const int64_t n = counts[r];
    if (n > 0) {
      const int per = v4 ? width / 4 : width;
      const unsigned bx = (unsigned)std::min<int64_t>(cdiv(n * per, 256), 4096);
      if (v4)
        hipLaunchKernelGGL(sparse_add_kernel<4>, dim3(bx), dim3(256), 0, s, shard, lo, elems, width, offs + pos,
                           rows + pos * width, n);
      else
        hipLaunchKernelGGL(sparse_add_kernel<1>, dim3(bx), dim3(256), 0, s, shard, lo, elems, width, offs + pos,
                           rows + pos * width, n);
      DCNR_LAUNCH_CHECK();
    }
    pos += n;
  }
  return DCNR_OK;
}

namespace {

template <int VEC, int NV>
void launch_sums(const EmbTabs& et, int nt, int64_t B, const EmbSortBufs& sb, const float* dx0,
                 int ld, const float* coef, int hps, int accumulate, hipStream_t s) {
  const int64_t n = (int64_t)nt * B, nseg = huge_segs(nt, B);
  float* hp = (float*)sb.tmp;
  const int wpb = ENT / WAVE;
  // head-position blocks, then one wave per HSEG segment: the long kernel's
  // extra waves write the huge-run pieces, the short kernel's add them up
  const dim3 gl((unsigned)(cdiv(n, (int64_t)ENT) + cdiv(nseg, (int64_t)wpb)));
  bool split = true;   // every column block of every table has >= NV groups
  for (int t = 0; t < nt; ++t) {
    const int G = et.width[t] / VEC, last = G % WAVE;
    if ((G < WAVE && G < NV) || (G >= WAVE && last != 0 && last < NV)) split = false;
  }
  if (split)
    hipLaunchKernelGGL((emb_runs_long_kernel<VEC, NV, true>), gl, dim3(ENT), 0, s, et, B, n,
                       sb.keys_s, sb.vals_s, dx0, ld, coef, hp, hps, nseg, accumulate);
  else
    hipLaunchKernelGGL((emb_runs_long_kernel<VEC, NV, false>), gl, dim3(ENT), 0, s, et, B, n,
                       sb.keys_s, sb.vals_s, dx0, ld, coef, hp, hps, nseg, accumulate);
  hipLaunchKernelGGL((emb_runs_short_kernel<VEC, NV>), gl, dim3(ENT), 0, s, et, nt, B,
                     sb.keys_s, sb.vals_s, dx0, ld, coef, hp, hps, nseg, accumulate);
}

template <int VEC>
void launch_sums_nv(int nv, const EmbTabs& et, int nt, int64_t B, const EmbSortBufs& sb,
                    const float* dx0, int ld, const float* coef, int hps, int accumulate,
                    hipStream_t s) {
  switch (nv) {
#define CASE(k) \
  case k: launch_sums<VEC, k>(et, nt, B, sb, dx0, ld, coef, hps, accumulate, s); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
  }
}

}  // namespace

dcnr_status emb_segment_sum(const EmbBwdDesc& e, const EmbSortBufs& sb, int64_t B,
                            const float* dx0, int ld, const float* coef, int accumulate,
                            hipStream_t s) {
  const int64_t n = (int64_t)e.n_tab * B;
  if (n <= 0) return DCNR_OK;
  if (e.nv < 1 || e.nv > 8) {
    set_error("embedding backward: %d cross basis vectors unsupported", e.nv);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  const int hps = huge_stride(e.width, e.n_tab);
  if ((size_t)huge_segs(e.n_tab, B) * 2 * hps * 4 > sb.tmp_bytes) {
    set_error("embedding backward: sort scratch too small for the huge-run pieces");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  const EmbTabs et = make_tabs(e);
  if (vec4_ok(e, dx0, ld))
    launch_sums_nv<4>(e.nv, et, e.n_tab, B, sb, dx0, ld, coef, hps, accumulate, s);
  else
    launch_sums_nv<1>(e.nv, et, e.n_tab, B, sb, dx0, ld, coef, hps, accumulate, s);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
