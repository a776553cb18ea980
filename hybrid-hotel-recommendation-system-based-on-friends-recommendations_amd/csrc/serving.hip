// The steps either side of scoring in /recommendations (main.py:294-357), on
// the device, for candidate sets of up to SV_MAX items:
//
//   candidate union   _generate_candidates, main.py:196-203: the positive
//                     hotels plus the neighbours the cosine index returns for
//                     each (position 0 dropped), as a set (here: ascending ids)
//   ranking batch     preprocess_for_ranking, main.py:215-230: the user id
//                     repeated, and each candidate's item id, categorical codes
//                     and scaled numeric features gathered from per-item tables
//   rank by score     sorted(zip(scores, ids), key=score, reverse=True),
//                     main.py:325: descending, equal scores keep input order
//   MMR re-rank       rerank_with_mmr, main.py:133-169: greedy
//                     argmax of lambda * score - (1 - lambda) * max cosine
//                     similarity to the already selected items
//
// Each is one workgroup (the sets are tens to thousands of items): the sort is
// an LDS bitonic sort of (key, position) pairs, so ties resolve by position
// exactly as Python's stable sort does.
#include "dcnr_internal.h"

#include <cfloat>
#include <climits>

namespace dcnr {
namespace {

constexpr int SV_NT = 1024;
constexpr int SV_MAX = 4096;   // max candidates per call (LDS sort capacity)
constexpr size_t MMR_LDS_MAX = 152 * 1024;   // dynamic LDS of mmr_lds_kernel (+ ~4 KiB static)

// ascending bitonic sort of n2 (power of two) (key, val) pairs in LDS;
// less(a, b) on (key, val)
template <typename K>
__device__ void lds_bitonic(K* key, int* val, int n2) {
  for (int k2 = 2; k2 <= n2; k2 <<= 1) {
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += SV_NT) {
        const int lo = ((t & ~(j - 1)) << 1) | (t & (j - 1));
        const int hi = lo + j;
        const bool asc = (lo & k2) == 0;
        const K ka = key[lo], kb = key[hi];
        const int va = val[lo], vb = val[hi];
        const bool b_less = kb < ka || (kb == ka && vb < va);
        if (asc ? b_less : !b_less && (ka != kb || va != vb)) {
          key[lo] = kb; key[hi] = ka; val[lo] = vb; val[hi] = va;
        }
      }
      __syncthreads();
    }
  }
}

// union of positives[Q] and idx[Q][k][1:] (rows < 0 skipped) -> ascending
// unique rows; out_count[0] = number of rows
__global__ __launch_bounds__(SV_NT) void union_kernel(const int64_t* pos, int64_t Q,
                                                      const int64_t* idx, int k, int64_t* out,
                                                      int32_t* out_count) {
  __shared__ int64_t key[SV_MAX];
  __shared__ int val[SV_MAX];
  __shared__ int wsum[SV_NT / 64];
  const int n = (int)(Q * k);   // positives + k-1 neighbours per query
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int t = threadIdx.x; t < n2; t += SV_NT) {
    int64_t r = INT64_MAX;
    if (t < n) {
      const int64_t q = t / k, j = t % k;
      r = j == 0 ? pos[q] : idx[q * k + j];
      if (r < 0) r = INT64_MAX;
    }
    key[t] = r;
    val[t] = t;
  }
  __syncthreads();
  lds_bitonic(key, val, n2);
  // compact the first occurrence of every id (ballot prefix per wave, wave
  // totals through LDS)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int running = 0;
  for (int base = 0; base < n2; base += SV_NT) {
    const int t = base + threadIdx.x;
    const bool f = t < n2 && key[t] != INT64_MAX && (t == 0 || key[t] != key[t - 1]);
    const uint64_t m = __ballot(f);
    const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int off = running, tot = 0;
    for (int i = 0; i < SV_NT / 64; ++i) {
      off += i < w ? wsum[i] : 0;
      tot += wsum[i];
    }
    if (f) out[off + pre] = key[t];
    running += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *out_count = running;
}

// ranking batch for one user: user_out[i] = user_row, item_out[i] = rows[i],
// cat_out[i][:] = item_cat[rows[i]][:], num_out[i][:] = item_num[rows[i]][:]
__global__ void batch_kernel(const int64_t* rows, int64_t n, int64_t user_row,
                             const int64_t* item_cat, int K, const float* item_num, int F,
                             int64_t n_items, int64_t* user_out, int64_t* item_out,
                             int64_t* cat_out, float* num_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.y + threadIdx.y;
  if (i >= n) return;
  int64_t r = rows[i];
  r = r < 0 ? 0 : (r >= n_items ? n_items - 1 : r);
  if (threadIdx.x == 0) { user_out[i] = user_row; item_out[i] = rows[i]; }
  for (int c = threadIdx.x; c < K; c += blockDim.x) cat_out[i * K + c] = item_cat[r * K + c];
  for (int c = threadIdx.x; c < F; c += blockDim.x) num_out[i * F + c] = item_num[r * F + c];
}

// order[i] = position of the i-th highest score (ties: lower position first)
__global__ __launch_bounds__(SV_NT) void rank_kernel(const float* scores, int n, int64_t* order) {
  __shared__ float key[SV_MAX];
  __shared__ int val[SV_MAX];
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int t = threadIdx.x; t < n2; t += SV_NT) {
    key[t] = t < n ? -scores[t] : FLT_MAX;   // ascending on -score
    val[t] = t < n ? t : INT_MAX;
  }
  __syncthreads();
  lds_bitonic(key, val, n2);
  for (int t = threadIdx.x; t < n; t += SV_NT) order[t] = val[t];
}

// block argmax of (v, -pos): highest v, lowest position on ties
__device__ void block_argmax(float v, int p, float* sv, int* sp, float& bv, int& bp) {
  // wave level
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int op = __shfl_xor(p, o, 64);
    if (ov > v || (ov == v && op < p)) { v = ov; p = op; }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { sv[w] = v; sp[w] = p; }
  __syncthreads();
  bv = sv[0];
  bp = sp[0];
  for (int i = 1; i < SV_NT / 64; ++i)
    if (sv[i] > bv || (sv[i] == bv && sp[i] < bp)) { bv = sv[i]; bp = sp[i]; }
  __syncthreads();
}

// Greedy MMR over n candidates in ranked order (rerank_with_mmr, main.py:133-169).
// rows[i] = embedding row of candidate i or -1 (no embedding: never picked
// after the first, contributes no similarity).  sim = cosine similarity
// (zero-norm rows -> 0, as sklearn's normalize + dot).  The first candidate is
// always taken; then up to min(top_k, n) - 1 more while some candidate is
// eligible.  Max-similarity is 0 while no selected item has an embedding.
__global__ __launch_bounds__(SV_NT) void mmr_kernel(const float* table, const float* inv, int d,
                                                    const int64_t* rows, const float* scores,
                                                    int n, float lambda, int top_k,
                                                    int64_t* out_pos, int32_t* out_count) {
  __shared__ float maxsim[SV_MAX];
  __shared__ unsigned char taken[SV_MAX];
  __shared__ float sv[SV_NT / 64];
  __shared__ int sp[SV_NT / 64];
  __shared__ float selv[256];
  __shared__ int any_sel;
  for (int t = threadIdx.x; t < n; t += SV_NT) { maxsim[t] = -FLT_MAX; taken[t] = 0; }
  if (threadIdx.x == 0) { any_sel = 0; taken[0] = 1; out_pos[0] = 0; }
  __syncthreads();
  const int want = min(top_k, n);
  int cnt = 1, last = 0;
  for (;;) {
    // fold the last selected item into every candidate's max similarity
    const int64_t sr = rows[last];
    if (sr >= 0) {
      const float is = inv[sr];
      for (int t = threadIdx.x; t < d; t += SV_NT) selv[t] = table[sr * d + t] * is;
      __syncthreads();
      for (int t = threadIdx.x; t < n; t += SV_NT) {
        const int64_t r = rows[t];
        if (r < 0 || taken[t]) continue;
        float s = 0.f;
        for (int c = 0; c < d; ++c) s += table[r * d + c] * selv[c];
        s *= inv[r];
        maxsim[t] = fmaxf(maxsim[t], s);
      }
      if (threadIdx.x == 0) any_sel = 1;
      __syncthreads();
    }
    if (cnt >= want) break;
    float v = -FLT_MAX;
    int p = INT_MAX;
    const bool sel = any_sel != 0;
    for (int t = threadIdx.x; t < n; t += SV_NT) {
      if (taken[t] || rows[t] < 0) continue;
      const float m = lambda * scores[t] - (1.f - lambda) * (sel ? maxsim[t] : 0.f);
      if (p == INT_MAX || m > v || (m == v && t < p)) { v = m; p = t; }
    }
    float bv;
    int bp;
    block_argmax(v, p, sv, sp, bv, bp);
    if (bp == INT_MAX) break;
    if (threadIdx.x == 0) { taken[bp] = 1; out_pos[cnt] = bp; }
    __syncthreads();
    ++cnt;
    last = bp;
  }
  for (int t = threadIdx.x + cnt; t < top_k; t += SV_NT) out_pos[t] = -1;
  if (threadIdx.x == 0) *out_count = cnt;
}

// The same greedy MMR with everything a selection round touches on chip:
// the candidates' raw rows (stride d+1: one row per thread, conflict-free)
// and inverse norms in LDS, each thread's candidates (t = tid + j*SV_NT) --
// validity, score, max similarity, taken -- in registers, so a round is one
// dot product per candidate and a block argmax (its two barriers), with no
// global loads.  Arithmetic as in mmr_kernel: s = sum_c row[c] * (sel[c] * is)
// in c order, then * inv.
__global__ __launch_bounds__(SV_NT) void mmr_lds_kernel(const float* table, const float* inv, int d,
                                                    const int64_t* rows, const float* scores,
                                                    int n, float lambda, int top_k,
                                                    int64_t* out_pos, int32_t* out_count) {
  constexpr int MR = SV_MAX / SV_NT;   // candidates per thread
  __shared__ float sv[SV_NT / 64];
  __shared__ int sp[SV_NT / 64];
  __shared__ unsigned char vld[SV_MAX];
  extern __shared__ float lds_rows[];
  float* invs = lds_rows + (size_t)n * (d + 1);
  for (int e = threadIdx.x; e < n * d; e += SV_NT) {
    const int t = e / d, c = e - t * d;
    const int64_t r = rows[t];
    lds_rows[t * (d + 1) + c] = r >= 0 ? table[r * d + c] : 0.f;
  }
  bool ok[MR], tk[MR];
  float sc[MR], ms[MR];
#pragma unroll
  for (int j = 0; j < MR; ++j) {
    const int t = threadIdx.x + j * SV_NT;
    const int64_t r = t < n ? rows[t] : -1;
    ok[j] = r >= 0;
    tk[j] = t == 0;
    sc[j] = t < n ? scores[t] : 0.f;
    ms[j] = -FLT_MAX;
    if (t < n) {
      invs[t] = r >= 0 ? inv[r] : 0.f;
      vld[t] = r >= 0;
    }
  }
  if (threadIdx.x == 0) out_pos[0] = 0;
  __syncthreads();
  const int want = min(top_k, n);
  int cnt = 1, last = 0;
  bool sel = false;
  for (;;) {
    // fold the last selected item into every candidate's max similarity
    if (vld[last]) {
      const float is = invs[last];
      const float* sr = lds_rows + last * (d + 1);
#pragma unroll
      for (int j = 0; j < MR; ++j) {
        const int t = threadIdx.x + j * SV_NT;
        if (t >= n || !ok[j] || tk[j]) continue;
        const float* rw = lds_rows + t * (d + 1);
        float s = 0.f;
        for (int c = 0; c < d; ++c) s += rw[c] * (sr[c] * is);
        s *= invs[t];
        ms[j] = fmaxf(ms[j], s);
      }
      sel = true;
    }
    if (cnt >= want) break;
    float v = -FLT_MAX;
    int p = INT_MAX;
#pragma unroll
    for (int j = 0; j < MR; ++j) {
      const int t = threadIdx.x + j * SV_NT;
      if (t >= n || tk[j] || !ok[j]) continue;
      const float m = lambda * sc[j] - (1.f - lambda) * (sel ? ms[j] : 0.f);
      if (p == INT_MAX || m > v || (m == v && t < p)) { v = m; p = t; }
    }
    float bv;
    int bp;
    block_argmax(v, p, sv, sp, bv, bp);
    if (bp == INT_MAX) break;
    if (bp % SV_NT == (int)threadIdx.x) tk[bp / SV_NT] = true;   // the owner thread
    if (threadIdx.x == 0) out_pos[cnt] = bp;
    ++cnt;
    last = bp;
  }
  for (int t = threadIdx.x + cnt; t < top_k; t += SV_NT) out_pos[t] = -1;
  if (threadIdx.x == 0) *out_count = cnt;
}

// Batch assembly of a device-resident dataset (the DataLoader of
// train.py:195-196): dst_a[i] = src_a[idx[i]] for each array a, whole rows of
// row_bytes (a multiple of 4) copied as dwords, one wave per (row, array).
struct RowGather {
  const char* src[8];
  char* dst[8];
  int64_t row_bytes[8];
  int n;
};

__global__ __launch_bounds__(256) void gather_rows_kernel(const int64_t* idx, int64_t n,
                                                          int64_t n_src, RowGather g) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= n * g.n) return;
  const int a = (int)(w % g.n);
  const int64_t i = w / g.n;
  int64_t r = idx[i];
  r = r < 0 ? 0 : (r >= n_src ? n_src - 1 : r);
  const int64_t words = g.row_bytes[a] >> 2;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(g.src[a] + r * g.row_bytes[a]);
  uint32_t* d = reinterpret_cast<uint32_t*>(g.dst[a] + i * g.row_bytes[a]);
  for (int64_t k = lane; k < words; k += 64) d[k] = s[k];
}

}  // namespace

dcnr_status gather_rows(const int64_t* idx, int64_t n, int64_t n_src, int n_arrays,
                        const void* const* src, void* const* dst, const int64_t* row_bytes,
                        hipStream_t s) {
  if (n_arrays < 1 || n_arrays > 8 || n < 0 || n_src < 1) {
    set_error("gather_rows: 1..8 arrays, n_src >= 1");
    return DCNR_BAD_ARG;
  }
  RowGather g;
  g.n = n_arrays;
  for (int a = 0; a < n_arrays; ++a) {
    if (!src[a] || !dst[a] || row_bytes[a] <= 0 || row_bytes[a] % 4) {
      set_error("gather_rows: array %d: null pointer or row bytes %lld not a multiple of 4", a,
                (long long)row_bytes[a]);
      return DCNR_BAD_ARG;
    }
    g.src[a] = (const char*)src[a];
    g.dst[a] = (char*)dst[a];
    g.row_bytes[a] = row_bytes[a];
  }
  if (n == 0) return DCNR_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)cdiv(n * n_arrays, 4)), dim3(256), 0, s,
                     idx, n, n_src, g);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status candidate_union(const int64_t* pos, int64_t Q, const int64_t* idx, int k,
                            int64_t* out, int32_t* out_count, hipStream_t s) {
  if (Q < 0 || k < 1 || Q * k > SV_MAX) {
    set_error("candidate_union: Q*k=%lld exceeds %d", (long long)(Q * k), SV_MAX);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  hipLaunchKernelGGL(union_kernel, dim3(1), dim3(SV_NT), 0, s, pos, Q, idx, k, out, out_count);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status ranking_batch(const int64_t* rows, int64_t n, int64_t user_row, const int64_t* item_cat,
                          int K, const float* item_num, int F, int64_t n_items, int64_t* user_out,
                          int64_t* item_out, int64_t* cat_out, float* num_out, hipStream_t s) {
  if (n <= 0) return DCNR_OK;
  dim3 blk(16, 16);
  hipLaunchKernelGGL(batch_kernel, dim3((unsigned)cdiv(n, 16)), blk, 0, s, rows, n, user_row,
                     item_cat, K, item_num, F, n_items, user_out, item_out, cat_out, num_out);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status rank_desc(const float* scores, int64_t n, int64_t* order, hipStream_t s) {
  if (n > SV_MAX) {
    set_error("rank_by_score: n=%lld exceeds %d", (long long)n, SV_MAX);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (n <= 0) return DCNR_OK;
  hipLaunchKernelGGL(rank_kernel, dim3(1), dim3(SV_NT), 0, s, scores, (int)n, order);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status mmr_rerank(const float* table, const float* inv, int d, const int64_t* rows,
                       const float* scores, int64_t n, float lambda, int top_k, int64_t* out_pos,
                       int32_t* out_count, hipStream_t s) {
  if (n > SV_MAX || d > 256 || d < 1 || top_k < 1) {
    set_error("mmr_rerank: n=%lld (max %d), d=%d (max 256), top_k=%d", (long long)n, SV_MAX, d,
              top_k);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (n <= 0) return DCNR_OK;
  // candidate rows staged in LDS when they fit (the same arithmetic, in the
  // same order, as the kernel that re-reads them from the table)
  const size_t lds = ((size_t)n * (d + 1) + (size_t)n) * sizeof(float);
  if (lds <= MMR_LDS_MAX) {
    TRY_ST(set_max_dyn_lds((const void*)mmr_lds_kernel, MMR_LDS_MAX));
    hipLaunchKernelGGL(mmr_lds_kernel, dim3(1), dim3(SV_NT), lds, s, table, inv, d, rows, scores, (int)n,
                       lambda, top_k, out_pos, out_count);
  } else {
    hipLaunchKernelGGL(mmr_kernel, dim3(1), dim3(SV_NT), 0, s, table, inv, d, rows, scores, (int)n,
                       lambda, top_k, out_pos, out_count);
  }
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
