// Internal declarations shared by the libdcnr HIP translation units.
// gfx950 (MI355X / CDNA4) only: 64-lane waves, MFMA, 160 KiB LDS per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>

#include <algorithm>
#include <cmath>

#include "../../include/dcnr.h"

namespace dcnr {

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int WAVE = 64;

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
// Raise a kernel's dynamic-LDS limit to at least `bytes` on the current
// device: thread-safe and per device (the serving path runs the eval forward
// from several host threads; one process may drive several devices).
dcnr_status set_max_dyn_lds(const void* kernel, size_t bytes);
#define DCNR_HIP(call)                                                              \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::dcnr::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return DCNR_HIP_ERROR;                                                        \
    }                                                                               \
  } while (0)
#define TRY_ST(x)                         \
  do {                                    \
    dcnr_status st_ = (x);                \
    if (st_ != DCNR_OK) return st_;       \
  } while (0)

#define DCNR_LAUNCH_CHECK()                                                         \
  do {                                                                              \
    hipError_t e_ = hipGetLastError();                                              \
    if (e_ != hipSuccess) {                                                         \
      ::dcnr::set_error("%s:%d launch: %s", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return DCNR_HIP_ERROR;                                                        \
    }                                                                               \
  } while (0)

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t rup(int64_t a, int64_t b) { return cdiv(a, b) * b; }

// ------------------------------------------------------------- storage T
template <typename T> struct St;
template <> struct St<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct St<bf16> {
  static __device__ __forceinline__ float ld(const bf16* p) { return (float)(*p); }
  static __device__ __forceinline__ void st(bf16* p, float v) { *p = (bf16)v; }
};

// ------------------------------------------------ buffer loads / hand-off
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

// LDS-DMA of 16 B per lane into lds_dst + 16 * lane (lds_dst wave-uniform),
// from byte offset `off` of the buffer (an out-of-range offset writes 0).
// Inline asm on purpose: hipcc tracks builtin LDS-DMAs as pending LDS writes
// and drains them (vmcnt(0)) before every ds_read, which would serialise a stage ring;
// the caller's counted vmcnt waits are the only synchronisation.
// M0 (compiler-reserved) is an input operand ("{m0}"): the compiler sets it
// before the statement and knows it changed -- no save / restore inside the
// asm, which cost the fused tower 3 % (profiles/lab/r05_tower_ablation.txt).
// (Default cache policy: the nt policy measured 4.06 -> 4.17 ms per step,
// profiles/lab/r03ae_dma_nt_ab.txt.)
__device__ __forceinline__ void dma16(u32x4 rsrc, int off, uint32_t lds_dst) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, 0 offen lds"
      :
      : "v"(off), "s"(rsrc), "{m0}"(lds_dst)
      : "memory");
}

// dma16's form with the uniform part of the offset in an SGPR (soff): a
// stream of pieces then costs one VGPR per lane pattern however many pieces
// a wave issues.
__device__ __forceinline__ void dma16s(u32x4 rsrc, int voff, int soff, uint32_t lds_dst) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %3 offen lds"
      :
      : "v"(voff), "s"(rsrc), "{m0}"(lds_dst), "s"(soff)
      : "memory");
}

__device__ __forceinline__ u32x4 rsrc_words(const void* p, int64_t bytes) {
  const uint64_t a = (uint64_t)p;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xFFFFu, p ? (uint32_t)bytes : 0u, 0x00020000u};
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

constexpr int OOR = 0x7fffff00;  // a buffer offset past num_records: loads 0, stores dropped

// Raw buffer descriptor over [p, p + bytes) (bytes < 2^31).  Out-of-range
// offsets load 0 with no branch, so unrolled load batches stay branch-free.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, p ? (int)bytes : 0, 0x00020000);
}

// Split-reduction hand-off (cdna_hip_programming.md, "In-launch split-K
// reduction"): every block stores its partial with plain stores and calls
// this; it returns true in exactly one block, the last arriver, which may
// then read all partials with plain loads.  `flag` is an int in the block's
// LDS.  The counter is zero at rest (re-zeroed by the last arriver; zeroed
// per forward by pack_all before first use).
__device__ __forceinline__ bool last_arriver(int* counter, int n_arrivals, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int prev = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = prev == n_arrivals - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// ReLU (train.py:117, 122) with one NaN rule for every path: max over the
// value's bits as a signed integer, which is what the fused eval tower's
// packed-int16 max on the bf16 activation does (tower.hip) -- +NaN (the NaN
// arithmetic yields here) and +inf pass, as torch.relu passes NaN; -0, -inf
// and a negative-signed NaN give +0.  (fmaxf would map every NaN to 0.)
__device__ __forceinline__ float relu_f(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

// BatchNorm backward apply (train.py:225 through nn.BatchNorm1d, train
// mode): dt = k0 du - k1 xhat - k2, xhat = (t - mean) invstd, with the
// per-column k0 = gamma invstd, k1, k2 from the batch sums.  One fixed
// operation order for the row passes (Bwd*ApplyOp) and the dX GEMM's fused
// operand transform (gemm_ws.hip), so the two give the same bits.
__device__ __forceinline__ float bn_bwd_dt(float u, float t, float mu, float is, float k0, float k1,
                                           float k2) {
  const float xh = (t - mu) * is;
  return fmaf(-k1, xh, k0 * u) - k2;
}

// The weight gradient's split-K combine, one 64 k x 16 n tile of
// out[n][k] (+)= sum_z slab[z][k][n] by 256 threads (splitk_reduce_t's
// kernel, and gemm_dw's tail when it combines the previous call's slab):
// sum in fixed z order into LDS t, barrier, transposed store of rows of out.
constexpr int RT_K = 64, RT_N = 16;
template <bool NT = false>
__device__ __forceinline__ void splitk_t_sum(const float* slab, int splits, int64_t stride, int ld, int N,
                                             int K, int bx, int by, int idx, float (*t)[RT_N + 1]) {
  const int k0 = bx * RT_K, n0 = by * RT_N;
  const int kk = idx >> 2, nq = idx & 3;
  const int k = k0 + kk, n = n0 + 4 * nq;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k < K && n < N) {
    const float* base = slab + (int64_t)k * ld + n;
    int z = 0;
    for (; z + 16 <= splits; z += 16) {
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float4* pp = reinterpret_cast<const float4*>(base + (int64_t)(z + u) * stride);
        if constexpr (NT) {
          typedef float f4v __attribute__((ext_vector_type(4)));
          const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(pp));
          v[u] = make_float4(w.x, w.y, w.z, w.w);
        } else {
          v[u] = *pp;
        }
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; z < splits; ++z) {
      const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)z * stride);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  t[kk][4 * nq] = s.x; t[kk][4 * nq + 1] = s.y; t[kk][4 * nq + 2] = s.z; t[kk][4 * nq + 3] = s.w;
}
__device__ __forceinline__ void splitk_t_store(int N, int K, float* out, int accumulate, int vec_out, int bx,
                                               int by, int idx, const float (*t)[RT_N + 1]) {
  const int k0 = bx * RT_K, n0 = by * RT_N;
  const int nn = idx >> 4, kq = idx & 15;
  const int n = n0 + nn, k = k0 + 4 * kq;
  if (n >= N) return;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = t[4 * kq + j][nn];
  float* o = out + (int64_t)n * K + k;
  if (vec_out && k + 3 < K) {
    float4 r = make_float4(v[0], v[1], v[2], v[3]);
    if (accumulate) {
      const float4 a = *reinterpret_cast<const float4*>(o);
      r.x += a.x; r.y += a.y; r.z += a.z; r.w += a.w;
    }
    *reinterpret_cast<float4*>(o) = r;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k + j < K) o[j] = accumulate ? o[j] + v[j] : v[j];
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- register-only wave reductions (no LDS crossbar round trips)
// gfx950 v_permlane32_swap / v_permlane16_swap exchange half-waves / rows;
// the last 16 lanes reduce with DPP (quad_perm, row_half_mirror, row_mirror).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_sum(float t) {   // sum over each 16-lane row, in every lane
  t += dpp<0xB1>(t);    // quad_perm [1,0,3,2]
  t += dpp<0x4E>(t);    // quad_perm [2,3,0,1]
  t += dpp<0x141>(t);   // row_half_mirror
  t += dpp<0x140>(t);   // row_mirror
  return t;
}
// full 64-lane sum of v, in every lane
__device__ __forceinline__ float wave_sum_dpp(float v) {
  const unsigned u = __float_as_uint(v);
  auto h = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  float t = __uint_as_float(h[0]) + __uint_as_float(h[1]);
  const unsigned ut = __float_as_uint(t);
  auto r = __builtin_amdgcn_permlane16_swap(ut, ut, false, false);
  t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  return row16_sum(t);
}
// two independent 64-lane sums at once (wave-uniform results)
__device__ __forceinline__ void wave_sum2(float a, float b, float& sa, float& sb) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  const float t = __uint_as_float(p[0]) + __uint_as_float(p[1]);     // lanes 0-31: a, 32-63: b
  const unsigned ut = __float_as_uint(t);
  auto r = __builtin_amdgcn_permlane16_swap(ut, ut, false, false);
  const float u = row16_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));  // rows: a, a, b, b
  sa = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), 0));
  sb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u), 32));
}
// four independent 64-lane sums at once (wave-uniform results)
__device__ __forceinline__ void wave_sum4(float a, float b, float c, float d, float& sa, float& sb,
                                          float& sc, float& sd) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(d), false, false);
  const float ab = __uint_as_float(p[0]) + __uint_as_float(p[1]);   // lanes 0-31: a, 32-63: b
  const float cd = __uint_as_float(q[0]) + __uint_as_float(q[1]);   // lanes 0-31: c, 32-63: d
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(ab), __float_as_uint(cd), false, false);
  const float t = row16_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));  // rows: a, c, b, d
  sa = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 0));
  sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 16));
  sb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 32));
  sd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 48));
}

// Counter-based dropout mask: 32 random bits per (seed, layer, row, column
// pair), deterministic, so backward regenerates the forward mask without
// storing it.  Column 2k uses the low 16 bits, 2k+1 the high 16 bits; an
// element is kept iff its 16 bits >= thresh16 = round(p * 65536), i.e. with
// probability 1 - p (to 2^-16).  Two murmur3 fmix32 rounds (32-bit integer
// ops only: ~8 VALU per element).
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16; x *= 0x85EBCA6Bu;
  x ^= x >> 13; x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t dropout_bits(uint64_t seed, int layer, int64_t row,
                                                 int colpair) {
  uint32_t x = fmix32((uint32_t)row * 0x9E3779B1u ^ (uint32_t)seed ^ ((uint32_t)layer * 0x7FEB352Du));
  return fmix32((x + (uint32_t)colpair * 0x846CA68Bu) ^ (uint32_t)(seed >> 32));
}

// y[v] *= keep(r, c+v) ? inv_keep : 0 for V consecutive columns (c even)
template <int V>
__device__ __forceinline__ void apply_dropout(uint64_t seed, int layer, int64_t r, int c,
                                              uint32_t thresh16, float inv_keep, float (&y)[V]) {
#pragma unroll
  for (int v = 0; v < V; v += 2) {
    const uint32_t bits = dropout_bits(seed, layer, r, (c + v) >> 1);
    y[v] = (bits & 0xFFFFu) >= thresh16 ? y[v] * inv_keep : 0.f;
    y[v + 1] = (bits >> 16) >= thresh16 ? y[v + 1] * inv_keep : 0.f;
  }
}

// the 16-bit keep threshold of dropout probability p (see dropout_bits)
inline uint32_t drop_thresh16(float p) {
  return (uint32_t)std::min(65536.0, std::floor((double)p * 65536.0 + 0.5));
}

// train-mode BatchNorm apply + ReLU (train.py:117-122) from the batch affine
// sc = gamma invstd, sh = beta - mean sc: relu(t sc + sh) and, for the
// residual block's output, relu(t sc + sh + x) -- one explicit fma order for
// every pass that makes or rebuilds them (BnReluDropOp, BnAddRelu(Head)Op,
// the backward's rebuild of h_R)
__device__ __forceinline__ float bn_fwd_relu(float t, float sc, float sh) { return relu_f(fmaf(t, sc, sh)); }
__device__ __forceinline__ float bn_fwd_add_relu(float t, float sc, float sh, float x) {
  return relu_f(fmaf(t, sc, sh) + x);
}

// ------------------------------------------------------------------ GEMM
// C[M,N] = A[M,K] . B[N,K]^T   (logical).  A_T: A stored [K][lda] (m fastest),
// else [M][lda] (k fastest).  B_T: B stored [K][ldb] (n fastest), else [N][ldb].
// K, lda, ldb, and (for A_T/B_T) M/N are multiples of 8; pad columns are 0.
enum GemmEpi : int {
  EPI_STORE = 0,        // out(T or f32) = acc + bias[n]  (bias may be null)
  EPI_STORE_RESID = 1,  // out = acc + resid[m*ldr+n]
  EPI_SPLITK = 2,       // f32 slab[split][m][n] = acc
};

struct GemmArgs {
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  const float* bias;
  const void* resid; int64_t ldr;
  int64_t M, N, K;
  int64_t k_per_split;   // split-K chunk (multiple of BK), = K when no split
  int64_t slab_stride;   // elements between split slabs (EPI_SPLITK)
  int out_f32;           // 1: C is float, 0: C is T
  int xcd_split;         // set by gemm(): 1-D grid with a split's tiles on one XCD
};

// precision 0 = fp32 (f32 MFMA), 1 = bf16 (bf16 MFMA).
dcnr_status gemm(int precision, bool a_t, bool b_t, int epi, const GemmArgs& a, int splits,
                 hipStream_t s);

struct BnFinal {   // per BN layer
  const float* gamma; const float* beta; float* rmean; float* rvar; int64_t* nbt;
  float* scale; float* shift;   // y = t*scale + shift  (N)
  float* mean; float* invstd;   // saved for backward
};
// N = padded width, Nr = real width (parameters have Nr entries; pads -> 0)
dcnr_status bn_finalize2(const double* sums, int N, int Nr, int train, const BnFinal& f,
                         hipStream_t s);
// eval (running-stat) finalize of up to 16 BN layers in one launch
struct BnEvalBatch { BnFinal f[16]; int n, N, Nr; };
dcnr_status bn_eval_finalize(const BnEvalBatch& b, hipStream_t s);
// Fused reduce + consumer (used when no SyncBN hook must see the sums)
enum RedMode : int { RED_BN_FWD = 0, RED_BN_BWD = 1, RED_BIAS = 2, RED_SUMS = 3 };
constexpr int RED_G = 32;          // chunk groups per column group
constexpr int RED_MAX_CGRP = 64;   // column groups of 64 -> N <= 4096
constexpr int CNT_SLOTS = 512;     // hand-off counters in the workspace (zeroed by pack_all)
struct RedFinal {
  int mode; int accumulate; double count;
  double* red2;                                // workspace [RED_G][3][N] fp64
  int* counter;                                // workspace [RED_MAX_CGRP], zero at rest
  double* sums;                                // RED_SUMS: [3][N] + count

  BnFinal f;                                   // RED_BN_FWD (train)
  const float* gamma; const float* invstd;     // RED_BN_BWD
  float* dgamma; float* dbeta; float* dwf; float* coef;
  float* dbias_pre;                            // Linear bias in front of the BN: grad = 0
  float* grad;                                 // RED_BIAS
  const float* shiftf;                         // f32 shift of the stats partials (or null)
};


constexpr float BN_EPS = 1e-5f;
constexpr double BN_MOM = 0.1;

// Consumer of reduced column sums v0, v1, v2 (fp64) of column n: BN forward
// statistics (+ running stats), BN backward coefficients and parameter
// gradients, a bias gradient, or the raw sums for a SyncBN hook.  K (when
// has_k) is the shift the partials were taken relative to.
__device__ inline void red_finalize(const RedFinal& rf, int n, int N, int Nr, double v0, double v1,
                                    double v2, bool has_k, double K) {
  const double cnt = rf.count;
  const bool real = n < Nr;
  if (has_k) {  // unshift
    v1 = v1 + 2.0 * K * v0 + cnt * K * K;
    v0 = v0 + cnt * K;
  }
  if (rf.mode == RED_SUMS) {  // raw sums for the SyncBN hook (+ count at [3N])
    rf.sums[n] = v0;
    rf.sums[N + n] = v1;
    rf.sums[2 * N + n] = v2;
    if (n == 0) rf.sums[3 * N] = cnt;
  } else if (rf.mode == RED_BN_FWD) {
    const BnFinal& f = rf.f;
    if (!real) {
      f.scale[n] = 0.f; f.shift[n] = 0.f; f.mean[n] = 0.f; f.invstd[n] = 0.f;
      return;
    }
    double mean = v0 / cnt;
    double var = v1 / cnt - mean * mean;
    if (var < 0) var = 0;
    f.rmean[n] = (float)((1.0 - BN_MOM) * (double)f.rmean[n] + BN_MOM * mean);
    f.rvar[n] = (float)((1.0 - BN_MOM) * (double)f.rvar[n] + BN_MOM * var * cnt / (cnt - 1.0));
    if (n == 0 && f.nbt) f.nbt[0] += 1;
    float inv = (float)(1.0 / sqrt(var + (double)BN_EPS));
    float sc = f.gamma[n] * inv;
    f.scale[n] = sc;
    f.shift[n] = f.beta[n] - (float)mean * sc;
    f.mean[n] = (float)mean;
    f.invstd[n] = inv;
  } else if (rf.mode == RED_BN_BWD) {
    // v0 = sum dy, v1 = sum dy*xhat, v2 = sum dz*out (deep half of dW_f)
    const float a = real ? rf.gamma[n] * rf.invstd[n] : 0.f;
    rf.coef[n] = a;
    rf.coef[N + n] = (float)((double)a * v1 / cnt);
    rf.coef[2 * N + n] = (float)((double)a * v0 / cnt);
    if (real) {
      rf.dgamma[n] = rf.accumulate ? rf.dgamma[n] + (float)v1 : (float)v1;
      rf.dbeta[n] = rf.accumulate ? rf.dbeta[n] + (float)v0 : (float)v0;
      if (rf.dwf) rf.dwf[n] = rf.accumulate ? rf.dwf[n] + (float)v2 : (float)v2;
      // the Linear bias in front of a train-mode BatchNorm has an exactly zero
      // gradient (sum_b dt = gamma*invstd*(sum du - sum du - sum(xhat)*..) = 0)
      if (rf.dbias_pre && !rf.accumulate) rf.dbias_pre[n] = 0.f;
    }
  } else {  // RED_BIAS
    if (real) rf.grad[n] = rf.accumulate ? rf.grad[n] + (float)v0 : (float)v0;
  }
}

// bf16 weight-stationary streaming GEMM (gemm_ws.hip): C[M,N] = X[M,K] W[N,K]^T
enum NtEpi : int {
  NT_EPI_BIAS = 0,    // C bf16 = acc + bias[n] (bias padded to N, may be null)
  NT_EPI_F32 = 1,     // C f32  = acc
  NT_EPI_RESID = 2,   // C bf16 = acc + R[m][n] (bf16)
  // epilogues that also emit BatchNorm column partials part[group][2][N]
  // (f32; one row per workgroup group, reduced by reduce_fused):
  NT_EPI_BIAS_STATS = 3,   // C = acc + bias; part = [sum(c - bias), sum((c - bias)^2)]
  NT_EPI_RESID_BN = 4,     // C = (acc + R) * [H > 0]; part = [sum c, sum c*xhat(T)]
  NT_EPI_DROP_BN = 5,      // C = acc * [H != 0] * hscale; part = [sum c, sum c*xhat(T)]
  // eval-mode BatchNorm folded into the epilogue (bn_scale /
  // bn_shift = the running-stat affine of bn_finalize2):
  NT_EPI_BN_RELU = 6,        // C = relu((acc + bias) * sc + sh)
  NT_EPI_BN_RESID_RELU = 7,  // C = relu((acc + bias) * sc + sh + R)
  // the eval forward's last block: no C; the deep head dot of the bf16-rounded
  // relu((acc + bias) * sc + sh + R) with wf, one partial per row per wave of
  // each column slice: headp[slice * 8 + wave][m] (summed by head_parts)
  NT_EPI_BN_RESID_RELU_HEAD = 8,
  // the train backward's G = dt1 W1 + du of block 0: C bf16 = acc + R[m][n];
  // part = [sum c, sum c^2] (c the stored value; component 0 is the initial
  // layer's bias gradient, reduced with RED_BIAS)
  NT_EPI_RESID_SUM = 9,
};
// (c is the stored bf16 value; xhat(T) = (T[m][n] - mean[n]) * invstd[n])
struct NtArgs {
  const bf16* X; int64_t ldx; int64_t M; int K;
  const bf16* W; int64_t ldw; int N;
  void* C; int64_t ldc;
  const float* bias;
  const void* R; int64_t ldr;
  float hscale;                                     // DROP_BN: 1/(1-p)
  const uint32_t* Hb; int64_t ldhb;                 // 1-bit keep mask (RESID_BN, DROP_BN): bit
                                                    // c%32 of word [m][c/32] = keep column c
  const bf16* T; int64_t ldt;                       // BN input for xhat
  const float* mean; const float* invstd;
  const float* bn_scale; const float* bn_shift;     // BN_RELU, BN_RESID_RELU(_HEAD)
  // eval BN from the running statistics (bn_rm != null): the kernel computes
  // scale / shift itself (bn_eval_multi_kernel's arithmetic) instead of reading
  // bn_scale / bn_shift
  const float* bn_g; const float* bn_b; const float* bn_rm; const float* bn_rv;
  const float* wf; float* headp; int64_t ldh;      // BN_RESID_RELU_HEAD (wf: Nr entries;
                                                    // headp rows ldh apart, ldh >= M)
  float* part;                                      // column partials (stats epilogues)
  int Nr;                                           // real columns (eval BN / head: N pads to 8)
  // operand transform (RESID_BN / DROP_BN, Tx != null): X holds a BatchNorm
  // backward's du, and the GEMM's operand is dt = bn_bwd_dt(du, Tx, xmean,
  // xinvstd, xcoef[0 / K / 2K]) per column of K, written to dt (row stride
  // ldx) for the weight gradient -- the row pass folded into the dX GEMM
  const bf16* Tx; const float* xmean; const float* xinvstd; const float* xcoef; bf16* dt;
  int nslices, groups; int64_t mtiles;   // filled by gemm_ws
};
bool gemm_ws_supported(int64_t K, int64_t N);
// the dX GEMMs' fused BatchNorm-backward operand transform (NtArgs.Tx)
bool gemm_ws_xbn_supported(int epi, int64_t K, int64_t N);
// the train forward's BIAS / BIAS_STATS epilogues at 256 < K <= 512: the
// pipelined one-wave-per-SIMD variant (gemm_wsp.hip), taken by gemm_ws
bool gemm_wsp_supported(int epi, int64_t K, int64_t N);
dcnr_status gemm_wsp(int epi, const NtArgs& a, hipStream_t s, int* nparts);
// nparts (stats epilogues): rows of part written (the nchunks of reduce_fused)
dcnr_status gemm_ws(int epi, const NtArgs& a, hipStream_t s, int* nparts = nullptr);
// head partials of NT_EPI_BN_RESID_RELU_HEAD: rows of headp written (0: unsupported shape)
int gemm_ws_head_parts(int64_t N);
inline bool nt_epi_stats(int epi) {
  return (epi >= NT_EPI_BIAS_STATS && epi <= NT_EPI_DROP_BN) || epi == NT_EPI_RESID_SUM;
}

// bf16 weight-gradient GEMM (gemm_dw.hip): slab[split][n][k] = sum over the
// split's batch rows of A[b][n] * B[b][k]; A = dY [Btot][lda], B = X [Btot][ldb]
struct DwArgs {
  const bf16* A; int64_t lda;
  const bf16* B; int64_t ldb;
  float* C; int64_t ldc; int64_t slab_stride;
  int64_t Btot, k_per_split;
  int N, K, splits;
  int tiles_n, tiles_k;            // filled by gemm_dw
  // the PREVIOUS call's split-K combine, in this launch's tail (rslab !=
  // null): out[rN][rK] (+)= sum of rsplits slabs of another buffer, the
  // splitk_reduce_t tiles dealt over the workgroups
  const float* rslab; int rsplits; int64_t rstride; int rld, rN, rK; float* rout; int racc;
};
bool gemm_dw_supported(int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t Btot);
// split count for ~wg_target workgroups (0: the default, one per CU)
int gemm_dw_splits(int64_t N, int64_t K, int64_t Btot);
dcnr_status gemm_dw(const DwArgs& a, hipStream_t s);

// ------------------------------------------------------------ elementwise
struct PackDesc {            // W [rows][cols] f32 -> dst T [rows_p][ld] (+ optional transpose)
  const float* src; void* dst; void* dst_t;
  int rows, cols, ld, ld_t;  // dst ld >= cols (pad 0), dst_t is [cols_p][ld_t] with ld_t >= rows
  int rows_p, cols_p;
  int f32;                   // 1: dst is f32 whatever the batch's precision (no transpose)
};
// ------------------------------------------------ fused eval deep tower
// (tower.hip) the eval forward's initial Linear + R ResBlocks + deep head dot
// in one persistent launch; activations stay in registers.
constexpr int MAX_RES_TW = 8;
struct TowerPack {                     // fp32 reference-layout parameters -> packed bf16 slices
  const float* W0; int D; const float* b0;
  const float* w1[MAX_RES_TW]; const float* b1[MAX_RES_TW]; const float* g1[MAX_RES_TW];
  const float* be1[MAX_RES_TW]; const float* rm1[MAX_RES_TW]; const float* rv1[MAX_RES_TW];
  const float* w2[MAX_RES_TW]; const float* b2[MAX_RES_TW]; const float* g2[MAX_RES_TW];
  const float* be2[MAX_RES_TW]; const float* rm2[MAX_RES_TW]; const float* rv2[MAX_RES_TW];
  const float* wf;                     // deep head weights (final_linear.weight[:H])
  int H, HT, R;                        // HT = H rounded up to 64 (set by tower_pack)
  char* out;                           // tower_ws_bytes(H, R)
  int* err;                            // optional: 64 ints zeroed (the gather's error word)
};
struct TowerArgs {
  const bf16* x0; int64_t ldx; int64_t M;   // x0 [M][ldx] bf16, columns >= Dp ignored
  int Dp, H, R;
  const char* wp; int64_t wp_bytes;          // tower_pack's output
  const float* zc; const float* bias;        // cross half of the head [M], final_linear.bias
  float* logits;
  const int* err; int* err_mirror;           // the call's error word -> its mirror (may be null)
  int ntiles;                                // (set by eval_tower)
};
bool tower_supported(int Dp, int H, int R);
int64_t tower_ws_bytes(int H, int R);
dcnr_status tower_pack(const TowerPack& p, hipStream_t s);
dcnr_status eval_tower(const TowerArgs& a, hipStream_t s);

constexpr int MAX_PACK = 20;
struct PackBatch { PackDesc d[MAX_PACK]; int n; };
dcnr_status pack_weights(int precision, const PackBatch& pb, hipStream_t s);

constexpr int MAX_TABLES = 66;           // user, item + up to 64 categorical tables
struct GatherDesc {
  const float* tab[MAX_TABLES];  // user, item, cat...
  int64_t rows[MAX_TABLES];
  int width[MAX_TABLES];
  int off[MAX_TABLES];           // first x0 column of the table
  int n_tab;                     // 2 + n_cat
  int n_num;
  int D;
};
struct CrossParams {
  const float* w[8];     // [D] each
  const float* b[8];     // [D]
  int L;
  const float* wf_cross; // final_linear.weight + H  ([D])
};

dcnr_status gather_cross_fwd(int precision, const GatherDesc& g, const CrossParams& cp,
                             const int64_t* user, const int64_t* item, const int64_t* cat,
                             const float* num, int64_t B, void* x0, int ldx, float* zc,
                             int* err, int check, hipStream_t s);

// 16-byte-lane forward (gather_cross.hip): any subset of x0 (fp32 or bf16),
// the cross output x_L (fp32, BASELINE configs[1]) and the head partial zc.
struct GcOut {
  float* cross;   // [B][ld_cross] fp32 x_L, or null
  void* x0;       // [B][ld_x0] fp32 or bf16, or null
  float* zc;      // [B] w_f[H:] . x_L, or null
  int ld_cross, ld_x0;
  float* sc;      // [B][2L+1] per-sample cross scalars for the backward, or null:
                  // s_l = x_l . w_l (l < L), u_m = x_0 . w_m (m < L), u_f = x_0 . w_f[H:]
};
dcnr_status gather_cross_out(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                             const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                             const GcOut& o, int x0_bf16, int* err, int check, hipStream_t s);

// low-rank cross backward (cross_bwd.hip)
struct CrossGrads {
  float* dw[8]; float* db[8];      // cross_network.{l}.w.weight / .b grads [D]
  float* dwf_cross;                // grad final_linear.weight + H  [D]
  float* dbf;                      // grad final_linear.bias        [1]
};
size_t cross_bwd_scratch_bytes(int D, int L, int64_t B);
// sc: the forward's GcOut::sc; x0: the forward's stored x0 ([B][ldx], bf16 if
// x0_bf16); coef, alpha: [B][L+1] outputs (coef = dx0_cross coefficients on
// w_0..w_{L-1}, w_f[H:], read by emb_segment_sum)
dcnr_status cross_backward(const CrossParams& cp, int D, const float* sc, const float* dz,
                           const void* x0, int x0_bf16, int ldx, int64_t B, const CrossGrads& gr,
                           float* coef, float* alpha, void* scratch, size_t scratch_bytes,
                           int accumulate, hipStream_t s);

// deterministic embedding gradients (embed_bwd.hip)
struct EmbBwdDesc {
  float* grad[MAX_TABLES];       // dense grads, [rows][width] each
  int64_t rows[MAX_TABLES];
  int width[MAX_TABLES];
  int off[MAX_TABLES];           // first x0 column of the table
  int n_tab;
  const float* V[8];             // dx0_cross = sum_k coef[b][k] V[k] (w_0..w_{L-1}, w_f[H:])
  int nv;                        // L + 1
  uint8_t* touched;              // null, or a byte per sort key (row): set to 1 for each row written
};
struct EmbSortBufs {
  uint32_t *ids;                 // [n_tab * B] clamped ids, table-major
  uint32_t *keys, *vals;         // [n_tab * B] level-1 sorted (tables of > 1024 rows)
  uint32_t *keys_s, *vals_s;     // sorted
  void* tmp; size_t tmp_bytes;   // sort counts / offsets, then the huge-run pieces
};
size_t emb_sort_tmp_bytes(const int64_t* rows, const int* width, int n_tab, int64_t B);
dcnr_status emb_sort(const EmbBwdDesc& e, const int64_t* user, const int64_t* item,
                     const int64_t* cat, int64_t B, const EmbSortBufs& sb, hipStream_t s);
// distinct touched rows of tables `tabs` from the sorted keys (dcnr_emb_touched_rows)
struct TouchedArgs {
  int n;                         // tables asked for
  int tab[MAX_TABLES];           // their indices
  uint32_t base[MAX_TABLES];     // first sort key of each (sum of earlier tables' rows)
  int width[MAX_TABLES];
  int64_t elem_off[MAX_TABLES];
  int64_t shard;                 // owner = offset / shard
  int world;
};
dcnr_status emb_touched_rows(const TouchedArgs& a, const EmbSortBufs& sb, int64_t B, int64_t* out,
                             int64_t* table_counts, int64_t* owner_counts, hipStream_t s);
// the data-parallel sparse exchange's device halves (embed_bwd.hip): pack the
// touched rows (+ their offsets) into the all_to_all send buffer; add what
// each source rank sent into the owner's shard, sources in order
dcnr_status sparse_pack(const float* grad, const int64_t* offs, int64_t ld, const int64_t* tcnt,
                        int n_tables, int width, int64_t* out_off, float* out_rows, hipStream_t s);
dcnr_status sparse_accumulate(float* shard, int64_t lo, int64_t elems, int width, const int64_t* offs,
                              const float* rows, const int64_t* counts, int n_sources, hipStream_t s);
// grad row r of table t = sum over its samples of dx0_deep[b][off_t:off_t+w_t]
// + sum_k (sum over its samples of coef[b][k]) V[k][off_t:off_t+w_t]
dcnr_status emb_segment_sum(const EmbBwdDesc& e, const EmbSortBufs& sb, int64_t B,
                            const float* dx0_deep, int ld, const float* coef, int accumulate,
                            hipStream_t s);


// Column reductions: partial sums per row-chunk, part[nchunks][NK][N] (f32),
// reduced in fixed order into sums[3][N] (f64; components >= NK zeroed) with
// the row count at sums[3N] (the slot a SyncBN all-reduce also sums).
dcnr_status col_stats(int precision, const void* t, int64_t B, int N, int ld, float* part,
                      int* nchunks, hipStream_t s);                  // NK=2: t, t^2
dcnr_status col_sum(int precision, const void* x, int64_t B, int N, int ld, float* part,
                    int* nchunks, hipStream_t s);                    // NK=1
// (col_stats partials are shifted by K = t[0][n]; reduce_fused unshifts them.)

dcnr_status reduce_fused(int precision, const float* part, int nchunks, int NK, int N, int Nr,
                         const void* shift, const RedFinal& rf, hipStream_t s);
// coef[3][N] for dt = coef0*dy - coef1*xhat - coef2
dcnr_status bn_bwd_coef(const double* sums, int N, int Nr, const float* gamma, const float* invstd,
                        float* coef, int train, hipStream_t s);

// a = dropout(relu(t*scale+shift)); bits (bf16 only, may be null): the 1-bit
// image [B][ld/8 bytes] of a != 0 (bit c%8 of byte c/8 of the row)
dcnr_status bn_relu_drop(int precision, const void* t, void* a, int64_t B, int N, int ld,
                         const float* scale, const float* shift, float p, uint64_t seed,
                         int layer, hipStream_t s, uint8_t* bits = nullptr);
// out = relu(t*scale + shift + x); bits: the 1-bit image of out > 0
dcnr_status bn_add_relu2(int precision, const void* t, const void* x, void* out, int64_t B, int N,
                         int ld, const float* scale, const float* shift, hipStream_t s,
                         uint8_t* bits = nullptr);

// backward helpers -----------------------------------------------------
// du = g*[out>0], g = G[b,n] (G != null) or dz[b]*wf[n]; NK=3 partials:
// [du, du*xhat, dz*out] (xhat = (t-mean)*invstd; the 3rd only when G == null)
// (also writes du = g*[out>0] in the storage type)
// (G null and x non-null: the last block's out is rebuilt from t, x = the
// block input and the BN scale / shift sc, sh -- out is not read)
dcnr_status bwd_bn2_stats3(int precision, const void* G, const float* dz, const float* wf,
                           const void* out, const void* t, const float* mean, const float* invstd,
                           int64_t B, int N, int ld, void* du, float* part, int* nchunks,
                           hipStream_t s, const void* x = nullptr, const float* sc = nullptr,
                           const float* sh = nullptr);
// dt = coef0*du - coef1*xhat - coef2 (part/nchunks unused)
dcnr_status bwd_bn2_apply2(int precision, const void* du, const void* t, const float* mean,
                           const float* invstd, const float* coef, int64_t B, int N, int ld,
                           void* dt, float* part, int* nchunks, hipStream_t s);
// the same for the last block (g = dz (x) wf), bf16, du from the 1-bit
// [out > 0] image of the forward's head pass (bits [B][ld/8])
dcnr_status bwd_bn2_apply_rank1(const uint8_t* bits, const float* dz, const float* wf, const void* t,
                                const float* mean, const float* invstd, const float* coef,
                                int64_t B, int N, int ld, void* dt, hipStream_t s);
// dr = da * keep/(1-p) * [t*scale+shift > 0] (in place); NK=2 partials [dr, dr*xhat]
dcnr_status bwd_bn1_stats(int precision, void* da_dr, const void* t, const float* scale,
                          const float* shift, const float* mean, const float* invstd, int64_t B,
                          int N, int ld, float p, uint64_t seed, int layer, float* part,
                          int* nchunks, hipStream_t s);
// dt = coef0*dr - coef1*xhat - coef2 ; NK=1 partials of dt
dcnr_status bwd_bn1_apply2(int precision, const void* dr, const void* t, const float* mean,
                           const float* invstd, const float* coef, int64_t B, int N, int ld,
                           void* dt, float* part, int* nchunks, hipStream_t s);
// out[n] (+)= sums[n] as float, n < N
dcnr_status sums_to_grad(const double* sums, int N, float* out, int accumulate, hipStream_t s);
// out[n][k] (+)= sum_s slab[s][n][k]  (n < N, k < K; slab row stride ld_slab)
dcnr_status splitk_reduce(const float* slab, int splits, int64_t slab_stride, int ld_slab,
                          int N, int K, float* out, int accumulate, hipStream_t s);
// the same over transposed slabs [splits][K][ld] (gemm_dw.hip's layout):
// out[n][k] (+)= sum_z slab[z][k][n]
dcnr_status splitk_reduce_t(const float* slab, int splits, int64_t slab_stride, int ld_slab, int N,
                            int K, float* out, int accumulate, hipStream_t s);

// head
// last block + head fused: out = relu(BN2(t) + x); logits = out . wf[:Nr] + zc + bf
bool bn_add_relu_head_supported(int precision, int N);
dcnr_status bn_add_relu_head(int precision, const void* t, const void* x, void* out, int64_t B,
                             int N, int ld, const float* scale, const float* shift,
                             const float* wf, int Nr, const float* zc, const float* bf,
                             float* logits, hipStream_t s, uint8_t* bits = nullptr);
dcnr_status row_dot(int precision, const void* X, int ld, int N, const float* w, int64_t B,
                    float* out, hipStream_t s);
// logits[b] = sum_p part[p][b] (p = 0..np-1, fixed order) + zc[b] + bf
dcnr_status head_parts(const float* part, int np, const float* zc, const float* bf, int64_t B,
                       float* logits, hipStream_t s);
dcnr_status head_logits(const float* zdeep, const float* zc, const float* bf, int64_t B,
                        float* logits, hipStream_t s);
size_t bce_ws_bytes();
dcnr_status bce(const float* z, const float* y, int64_t B, float* loss, float* dz, float scale,
                double* part, hipStream_t s);

// optimizer
dcnr_status adam(int n, float* const* p, const float* const* g, float* const* m, float* const* v,
                 const int64_t* numel, float lr, float b1, float b2, float eps, float wd,
                 int64_t step, int decoupled, hipStream_t s,
                 const uint8_t* const* row_map = nullptr, const int32_t* row_width = nullptr);

// knn
dcnr_status row_inv_norms(const float* t, int64_t N, int d, float* out, hipStream_t s);
size_t topk_ws(int64_t N, int64_t Q, int k);
// k best of lists k-lists [lists][Q][k] by (dist, row as unsigned)
dcnr_status topk_merge(const float* dist, const int64_t* idx, int lists, int64_t Q, int k,
                       int64_t* out_idx, float* out_dist, hipStream_t s);
// tb: the bf16 copy from cosine_pack_rows, or nullptr (scan v4 then rounds
// the fp32 rows itself)
dcnr_status cosine_topk(const float* t, const float* inv, const bf16* tb, int64_t N, int d,
                        const float* q, int64_t Q, int k, int64_t* idx, float* dist, void* ws,
                        size_t ws_bytes, hipStream_t s);
dcnr_status cosine_pack_rows(const float* t, const float* inv, int64_t N, int d, bf16* out, hipStream_t s);

// serving (serving.hip)
dcnr_status gather_rows(const int64_t* idx, int64_t n, int64_t n_src, int n_arrays,
                        const void* const* src, void* const* dst, const int64_t* row_bytes,
                        hipStream_t s);
dcnr_status candidate_union(const int64_t* pos, int64_t Q, const int64_t* idx, int k,
                            int64_t* out, int32_t* out_count, hipStream_t s);
dcnr_status ranking_batch(const int64_t* rows, int64_t n, int64_t user_row, const int64_t* item_cat,
                          int K, const float* item_num, int F, int64_t n_items, int64_t* user_out,
                          int64_t* item_out, int64_t* cat_out, float* num_out, hipStream_t s);
dcnr_status rank_desc(const float* scores, int64_t n, int64_t* order, hipStream_t s);
dcnr_status mmr_rerank(const float* table, const float* inv, int d, const int64_t* rows,
                       const float* scores, int64_t n, float lambda, int top_k, int64_t* out_pos,
                       int32_t* out_count, hipStream_t s);

dcnr_status fill_zero(void* p, size_t bytes, hipStream_t s);
// *dst = *src with a system-scope store (dst may be pinned host memory)
dcnr_status mirror_word(const int* src, int* dst, hipStream_t s);
dcnr_status fill_zero_multi(int n, void* const* ptrs, const int64_t* bytes, hipStream_t s);

}  // namespace dcnr
