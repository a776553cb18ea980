// Row-major [B][ld] activation kernels of the deep tower: BatchNorm statistics,
// BN/ReLU/dropout application, residual add, and their backward.  All are HBM
// streams with 16-byte accesses (8 bf16 or 4 fp32 per thread), U rows in
// flight per thread (loads for U rows issued before any use), per-column
// constants held in registers, and column partial sums reduced
// deterministically (fixed order, fp64) -- no atomics.
//
// Reference semantics: ResBlock.forward (train.py:112-122), nn.BatchNorm1d
// (train: biased batch var for normalisation, running stats with momentum 0.1
// and unbiased var; eval: running stats), nn.ReLU, nn.Dropout.
// Batch variance is computed from sums shifted by the batch's first row
// (K = t[0]), so var = E[(t-K)^2] - E[t-K]^2 does not cancel when |mean| >> std.
#include "dcnr_internal.h"

#include <cmath>
#include <type_traits>

namespace dcnr {
namespace {

constexpr int NT = 256;
constexpr int UNROLL = 4;
// reduction passes: 2048 partial rows (8 blocks/CU in flight for HBM latency
// hiding); apply passes: 8192 short blocks (4096 / 16384 measured the same,
// 1024 / 512 reduction chunks slower: DESIGN.md section 8, round 2)
constexpr int TARGET_CHUNKS = 2048;
constexpr int APPLY_CHUNKS = 8192;

template <typename T> constexpr int VE = 16 / (int)sizeof(T);

template <typename T>
__device__ __forceinline__ void ldv(const T* p, float (&o)[VE<T>]) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  if constexpr (std::is_same<T, float>::value) {
    o[0] = __uint_as_float(u.x); o[1] = __uint_as_float(u.y);
    o[2] = __uint_as_float(u.z); o[3] = __uint_as_float(u.w);
  } else {
    const bf16* h = reinterpret_cast<const bf16*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)h[i];
  }
}
// NT: nontemporal store.  Measured per pass (cfg3): the forward BN applies
// run 8-12 % faster with it (their outputs are next read a layer later), the
// backward applies 14 % slower (dt is read right away by the dX and dW GEMMs).
template <typename T, bool NT = false>
__device__ __forceinline__ void stv(T* p, const float (&o)[VE<T>]) {
  uint4 u;
  if constexpr (std::is_same<T, float>::value) {
    u.x = __float_as_uint(o[0]); u.y = __float_as_uint(o[1]);
    u.z = __float_as_uint(o[2]); u.w = __float_as_uint(o[3]);
  } else {
    bf16* h = reinterpret_cast<bf16*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (bf16)o[i];
  }
  if constexpr (NT)
    __builtin_nontemporal_store(u32x4{u.x, u.y, u.z, u.w}, reinterpret_cast<u32x4*>(p));
  else
    *reinterpret_cast<uint4*>(p) = u;
}
template <int V>
__device__ __forceinline__ void ldc(const float* p, float (&o)[V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) o[v] = p[v];
}

// Generic row x column-group driver.  Each thread owns V consecutive columns
// (c0 = cg*V) and walks rows rsub, rsub+rpp, ... of its block's chunk, U rows
// per step (all loads first).  NK > 0: per-column partial sums per chunk.
// rows in flight per thread: UNROLL, or 2 for the bf16 BN apply / backward
// ops (several operands + per-column constants per row: at 4 rows they take
// 99-172 VGPRs, 2-4 waves/SIMD).  Same-box A/B (gpurun_out/r02r, r02s): the
// rowwise class 1.315 -> 1.226 ms/step, the step 4.21 -> 4.18 ms.
template <class Op> struct RowUnroll { static constexpr int v = UNROLL; };

template <typename T, int NK, class Op>
__global__ __launch_bounds__(NT) void rowcol_kernel(Op op, int64_t B, int N, int rows_per_chunk,
                                                    float* part) {
  constexpr int V = VE<T>;
  constexpr int UNROLL = RowUnroll<Op>::v;
  constexpr int NKA = NK > 0 ? NK : 1;
  const int tcols = (N + V - 1) / V;
  const int rpp = NT / tcols;
  const int rsub = threadIdx.x / tcols, cg = threadIdx.x % tcols;
  const int c0 = cg * V;
  float acc[NKA][V];
#pragma unroll
  for (int k = 0; k < NKA; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
  const int64_t r1 = min(B, r0 + rows_per_chunk);
  if (rsub < rpp) {
    typename Op::Cst cst;
    op.prep(c0, cst);
    for (int64_t r = r0 + rsub; r < r1; r += (int64_t)UNROLL * rpp) {
      typename Op::Reg q[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        int64_t rr = r + (int64_t)u * rpp;
        if (rr < r1) op.load(rr, c0, q[u]);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        int64_t rr = r + (int64_t)u * rpp;
        if (rr < r1) op.apply(rr, c0, cst, q[u], acc);
      }
    }
  }
  if constexpr (NK > 0) {
    __shared__ float red[NT * NK * V];
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int v = 0; v < V; ++v) red[(threadIdx.x * NK + k) * V + v] = acc[k][v];
    __syncthreads();
    if (rsub == 0) {
      for (int k = 0; k < NK; ++k)
        for (int v = 0; v < V; ++v) {
          int c = c0 + v;
          if (c >= N) continue;
          float s = 0.f;
          for (int rs = 0; rs < rpp; ++rs) s += red[((rs * tcols + cg) * NK + k) * V + v];
          part[((int64_t)blockIdx.x * NK + k) * N + c] = s;
        }
    }
  }
}

template <typename T, int NK, class Op>
dcnr_status run_rowcol(const Op& op, int64_t B, int N, float* part, int* nchunks, hipStream_t s) {
  constexpr int V = VE<T>;
  if (N % 8 || (N + V - 1) / V > NT) {
    set_error("rowcol: unsupported width %d", N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  // apply-only passes (no partials) take one short block per 16 rows (one
  // load round per thread); reduction passes keep TARGET_CHUNKS partial rows
  int rows = NK == 0 ? (int)std::max<int64_t>(16, cdiv(B, APPLY_CHUNKS))
                     : (int)std::max<int64_t>(32, cdiv(B, TARGET_CHUNKS));
  int nc = (int)cdiv(B, rows);
  if (nchunks) *nchunks = nc;
  if (B <= 0) return DCNR_OK;
  hipLaunchKernelGGL((rowcol_kernel<T, NK, Op>), dim3(nc), dim3(NT), 0, s, op, B, N, rows, part);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

struct NoCst {};

// ---------------------------------------------------------------- ops
// sums of (t-K) and (t-K)^2 with K = t[0] (the batch's first row)
template <typename T> struct StatsOp {
  const T* t; int ld;
  struct Cst { float k[VE<T>]; };
  struct Reg { float x[VE<T>]; };
  __device__ void prep(int c, Cst& q) const { ldv<T>(t + c, q.k); }
  __device__ void load(int64_t r, int c, Reg& q) const { ldv<T>(t + r * ld + c, q.x); }
  __device__ void apply(int64_t, int, const Cst& k, Reg& q, float (&acc)[2][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) {
      float d = q.x[v] - k.k[v];
      acc[0][v] += d;
      acc[1][v] += d * d;
    }
  }
};

template <typename T> struct ColSumOp {
  const T* x; int ld;
  typedef NoCst Cst;
  struct Reg { float a[VE<T>]; };
  __device__ void prep(int, Cst&) const {}
  __device__ void load(int64_t r, int c, Reg& q) const { ldv<T>(x + r * ld + c, q.a); }
  __device__ void apply(int64_t, int, const Cst&, Reg& q, float (&acc)[1][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) acc[0][v] += q.a[v];
  }
};

// 1-bit image of "stored value > 0" for V = 8 bf16 columns c..c+7 of row r
// (the keep mask the backward GEMM epilogues apply), one byte per thread
template <typename T>
__device__ __forceinline__ void store_pos_bits(uint8_t* bits, int64_t r, int ldb, int c,
                                               const float (&y)[VE<T>]) {
  if constexpr (sizeof(T) == 2) {
    uint32_t b = 0;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const uint16_t h = __builtin_bit_cast(uint16_t, (bf16)y[v]);
      b |= (uint32_t)((h & 0x7fffu) != 0 && !(h & 0x8000u)) << v;
    }
    bits[r * ldb + (c >> 3)] = (uint8_t)b;
  }
}

template <typename T> struct BnReluDropOp {  // a = dropout(relu(t*sc+sh))
  const T* t; T* a; int ld; const float* sc; const float* sh;
  float inv_keep; uint32_t thresh; uint64_t seed; int layer; int drop;
  uint8_t* bits;
  struct Cst { float sc[VE<T>], sh[VE<T>]; };
  struct Reg { float x[VE<T>]; };
  __device__ void prep(int c, Cst& q) const { ldc(sc + c, q.sc); ldc(sh + c, q.sh); }
  __device__ void load(int64_t r, int c, Reg& q) const { ldv<T>(t + r * ld + c, q.x); }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&)[1][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) q.x[v] = bn_fwd_relu(q.x[v], k.sc[v], k.sh[v]);
    if (drop) apply_dropout<VE<T>>(seed, layer, r, c, thresh, inv_keep, q.x);
    stv<T, true>(a + r * ld + c, q.x);
    if (bits) store_pos_bits<T>(bits, r, ld >> 3, c, q.x);
  }
};

template <typename T> struct BnAddReluOp {   // out = relu(t*sc+sh + x)
  const T* t; const T* x; T* out; int ld; const float* sc; const float* sh;
  uint8_t* bits;
  struct Cst { float sc[VE<T>], sh[VE<T>]; };
  struct Reg { float a[VE<T>], b[VE<T>]; };
  __device__ void prep(int c, Cst& q) const { ldc(sc + c, q.sc); ldc(sh + c, q.sh); }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(t + r * ld + c, q.a);
    ldv<T>(x + r * ld + c, q.b);
  }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&)[1][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) q.a[v] = bn_fwd_add_relu(q.a[v], k.sc[v], k.sh[v], q.b[v]);
    stv<T, true>(out + r * ld + c, q.a);
    if (bits) store_pos_bits<T>(bits, r, ld >> 3, c, q.a);
  }
};

// last residual block + head: out = relu(t*sc+sh + x) and, with a wave per
// row (N / V == 64 threads), logits[r] = out[r] . wf[:Nr] + zc[r] + bf
template <typename T> struct BnAddReluHeadOp {
  const T* t; const T* x; T* out; int ld; const float* sc; const float* sh;
  const float* wf; int Nr; const float* zc; const float* bf; float* logits;
  uint8_t* bits;   // train: 1-bit [out > 0] for the backward (null: none)
  struct Cst { float sc[VE<T>], sh[VE<T>], wf[VE<T>]; float bf; };
  struct Reg { float a[VE<T>], b[VE<T>]; };
  __device__ void prep(int c, Cst& q) const {
    ldc(sc + c, q.sc); ldc(sh + c, q.sh);
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) q.wf[v] = c + v < Nr ? wf[c + v] : 0.f;
    q.bf = bf[0];
  }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(t + r * ld + c, q.a);
    ldv<T>(x + r * ld + c, q.b);
  }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&)[1][VE<T>]) const {
    float d = 0.f;
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) {
      q.a[v] = bn_fwd_add_relu(q.a[v], k.sc[v], k.sh[v], q.b[v]);
      d += (float)(T)q.a[v] * k.wf[v];   // the stored (rounded) activation, as row_dot reads it
    }
    if (out) stv<T, true>(out + r * ld + c, q.a);   // (train: null, the backward rebuilds it)
    if (bits) store_pos_bits<T>(bits, r, ld >> 3, c, q.a);
    d = wave_sum_dpp(d);
    if ((threadIdx.x & 63) == 0) logits[r] = (d + zc[r]) + k.bf;
  }
};

// backward of out = relu(BN2(t2) + x): du = g*[out>0]; g = G or dz (x) wf.
// REBUILD (last block, g = dz (x) wf): `out` is the block input x and out is
// rebuilt as the head pass computed it, bf16(relu(t2*sc + sh + x)), so the
// forward never stores h_R
template <typename T, bool HAS_G, bool REBUILD = false> struct Bwd2StatsOp {
  const T* G; const float* dz; const float* wf; const T* out; const T* t;
  const float* mean; const float* invstd; int ld; T* du_out;
  const float* sc = nullptr; const float* sh = nullptr;
  struct Cst { float wf[VE<T>], mu[VE<T>], is[VE<T>], sc[REBUILD ? VE<T> : 1], sh[REBUILD ? VE<T> : 1]; };
  struct Reg { float o[VE<T>], t[VE<T>], g[VE<T>]; float d = 0.f; };
  __device__ void prep(int c, Cst& q) const {
    if (!HAS_G) ldc(wf + c, q.wf);
    ldc(mean + c, q.mu); ldc(invstd + c, q.is);
    if constexpr (REBUILD) { ldc(sc + c, q.sc); ldc(sh + c, q.sh); }
  }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(out + r * ld + c, q.o);
    ldv<T>(t + r * ld + c, q.t);
    if constexpr (HAS_G) ldv<T>(G + r * ld + c, q.g);
    else q.d = dz[r];
  }
  // du = g * [out > 0] is stored (storage type) and the sums use the stored
  // value, so the apply pass needs only du and t
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&acc)[3][VE<T>]) const {
    if constexpr (REBUILD) {
#pragma unroll
      for (int v = 0; v < VE<T>; ++v) q.o[v] = (float)(T)bn_fwd_add_relu(q.t[v], k.sc[v], k.sh[v], q.o[v]);
    }
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) {
      float g = HAS_G ? q.g[v] : q.d * k.wf[v];
      float du = (float)(T)(q.o[v] > 0.f ? g : 0.f);
      float xh = (q.t[v] - k.mu[v]) * k.is[v];
      acc[0][v] += du;
      acc[1][v] += du * xh;
      if (!HAS_G) acc[2][v] += q.d * q.o[v];
      q.g[v] = du;
    }
    stv<T>(du_out + r * ld + c, q.g);
  }
};
// dt2 = k0*du - k1*xhat - k2 (BN2 backward)
template <typename T> struct Bwd2ApplyOp {
  const T* du; const T* t; const float* mean; const float* invstd; const float* coef; int ld, N;
  T* dt;
  struct Cst { float mu[VE<T>], is[VE<T>], k0[VE<T>], k1[VE<T>], k2[VE<T>]; };
  struct Reg { float u[VE<T>], t[VE<T>]; };
  __device__ void prep(int c, Cst& q) const {
    ldc(mean + c, q.mu); ldc(invstd + c, q.is);
    ldc(coef + c, q.k0); ldc(coef + N + c, q.k1); ldc(coef + 2 * N + c, q.k2);
  }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(du + r * ld + c, q.u);
    ldv<T>(t + r * ld + c, q.t);
  }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&acc)[1][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) q.u[v] = bn_bwd_dt(q.u[v], q.t[v], k.mu[v], k.is[v], k.k0[v], k.k1[v], k.k2[v]);
    stv<T>(dt + r * ld + c, q.u);
  }
};
// last block (g = dz (x) wf, rank 1): dt2 = k0*du - k1*xhat - k2 with du
// rebuilt from dz, wf and the forward's 1-bit [out > 0] image (bf16), so the
// pass reads neither du nor out; du is the value Bwd2StatsOp stores, bit for bit
template <typename T> struct Bwd2ApplyRank1Op {
  const uint8_t* bits; const float* dz; const float* wf; const T* t; const float* mean;
  const float* invstd; const float* coef; int ld, N; T* dt;
  struct Cst { float mu[VE<T>], is[VE<T>], k0[VE<T>], k1[VE<T>], k2[VE<T>], wf[VE<T>]; };
  struct Reg { float t[VE<T>]; float d; uint32_t b; };
  __device__ void prep(int c, Cst& q) const {
    ldc(mean + c, q.mu); ldc(invstd + c, q.is); ldc(wf + c, q.wf);
    ldc(coef + c, q.k0); ldc(coef + N + c, q.k1); ldc(coef + 2 * N + c, q.k2);
  }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(t + r * ld + c, q.t);
    q.d = dz[r];
    q.b = bits[r * (ld >> 3) + (c >> 3)];
  }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&)[1][VE<T>]) const {
    float o[VE<T>];
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) {
      const float du = (q.b >> v) & 1u ? (float)(T)(q.d * k.wf[v]) : 0.f;
      o[v] = bn_bwd_dt(du, q.t[v], k.mu[v], k.is[v], k.k0[v], k.k1[v], k.k2[v]);
    }
    stv<T>(dt + r * ld + c, o);
  }
};

template <typename T> struct Bwd1StatsOp {
  T* da; const T* t; const float* sc; const float* sh; const float* mean; const float* invstd;
  int ld; float inv_keep; uint32_t thresh; uint64_t seed; int layer; int drop;
  struct Cst { float sc[VE<T>], sh[VE<T>], mu[VE<T>], is[VE<T>]; };
  struct Reg { float a[VE<T>], t[VE<T>]; };
  __device__ void prep(int c, Cst& q) const {
    ldc(sc + c, q.sc); ldc(sh + c, q.sh); ldc(mean + c, q.mu); ldc(invstd + c, q.is);
  }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(da + r * ld + c, q.a);
    ldv<T>(t + r * ld + c, q.t);
  }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&acc)[2][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) {
      float pre = fmaf(q.t[v], k.sc[v], k.sh[v]);
      q.a[v] = pre > 0.f ? q.a[v] : 0.f;
    }
    if (drop) apply_dropout<VE<T>>(seed, layer, r, c, thresh, inv_keep, q.a);
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) {
      float xh = (q.t[v] - k.mu[v]) * k.is[v];
      acc[0][v] += q.a[v];
      acc[1][v] += q.a[v] * xh;
    }
    stv<T>(da + r * ld + c, q.a);
  }
};

template <typename T> struct Bwd1ApplyOp {
  const T* dr; const T* t; const float* mean; const float* invstd; const float* coef; int ld, N;
  T* dt;
  struct Cst { float mu[VE<T>], is[VE<T>], k0[VE<T>], k1[VE<T>], k2[VE<T>]; };
  struct Reg { float a[VE<T>], t[VE<T>]; };
  __device__ void prep(int c, Cst& q) const {
    ldc(mean + c, q.mu); ldc(invstd + c, q.is);
    ldc(coef + c, q.k0); ldc(coef + N + c, q.k1); ldc(coef + 2 * N + c, q.k2);
  }
  __device__ void load(int64_t r, int c, Reg& q) const {
    ldv<T>(dr + r * ld + c, q.a);
    ldv<T>(t + r * ld + c, q.t);
  }
  __device__ void apply(int64_t r, int c, const Cst& k, Reg& q, float (&acc)[1][VE<T>]) const {
#pragma unroll
    for (int v = 0; v < VE<T>; ++v) q.a[v] = bn_bwd_dt(q.a[v], q.t[v], k.mu[v], k.is[v], k.k0[v], k.k1[v], k.k2[v]);
    stv<T>(dt + r * ld + c, q.a);
  }
};

// (1 / 4 rows in flight measured the same / slower: DESIGN.md section 8)
template <typename T, bool G, bool R> struct RowUnroll<Bwd2StatsOp<T, G, R>> { static constexpr int v = 2; };
template <typename T> struct RowUnroll<BnAddReluHeadOp<T>> { static constexpr int v = 2; };
template <typename T> struct RowUnroll<Bwd1ApplyOp<T>> { static constexpr int v = 2; };
template <typename T> struct RowUnroll<Bwd2ApplyOp<T>> { static constexpr int v = 2; };
template <typename T> struct RowUnroll<Bwd2ApplyRank1Op<T>> { static constexpr int v = 2; };
template <typename T> struct RowUnroll<BnAddReluOp<T>> { static constexpr int v = 2; };
template <typename T> struct RowUnroll<BnReluDropOp<T>> { static constexpr int v = 2; };

// ------------------------------------------------------------ small kernels
__global__ void bn_finalize_kernel(const double* sums, int N, int Nr, int train, BnFinal f) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  if (n >= Nr) {  // padded column: stays exactly zero
    f.scale[n] = 0.f; f.shift[n] = 0.f; f.mean[n] = 0.f; f.invstd[n] = 0.f;
    return;
  }
  double mean, var;
  if (train) {
    double cnt = sums[3 * N];
    mean = sums[n] / cnt;
    var = sums[N + n] / cnt - mean * mean;
    if (var < 0) var = 0;
    f.rmean[n] = (float)((1.0 - BN_MOM) * (double)f.rmean[n] + BN_MOM * mean);
    f.rvar[n] = (float)((1.0 - BN_MOM) * (double)f.rvar[n] + BN_MOM * var * cnt / (cnt - 1.0));
    if (n == 0 && f.nbt) f.nbt[0] += 1;
  } else {
    mean = f.rmean[n];
    var = f.rvar[n];
  }
  float inv = (float)(1.0 / sqrt(var + (double)BN_EPS));
  float sc = f.gamma[n] * inv;
  f.scale[n] = sc;
  f.shift[n] = f.beta[n] - (float)mean * sc;
  f.mean[n] = (float)mean;
  f.invstd[n] = inv;
}

// coef = [gamma*invstd, gamma*invstd*S1/cnt, gamma*invstd*S0/cnt] (train) or [gamma*invstd, 0, 0]
__global__ void bn_bwd_coef_kernel(const double* sums, int N, int Nr, const float* gamma,
                                   const float* invstd, float* coef, int train) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float a = n < Nr ? gamma[n] * invstd[n] : 0.f;
  coef[n] = a;
  if (train) {
    double cnt = sums[3 * N];
    coef[N + n] = (float)((double)a * sums[N + n] / cnt);
    coef[2 * N + n] = (float)((double)a * sums[n] / cnt);
  } else {
    coef[N + n] = 0.f;
    coef[2 * N + n] = 0.f;
  }
}

__global__ void sums_to_grad_kernel(const double* sums, int N, float* out, int accumulate) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float v = (float)sums[n];
  out[n] = accumulate ? out[n] + v : v;
}

// out[n][k] (+)= sum_z slab[z][n][k], z in fixed order.  Vector path (K and
// ld multiples of 4, 16-B aligned): 4 columns per lane, 16 slab loads in
// flight per lane; otherwise one element per lane.
__global__ void splitk_reduce_kernel(const float* slab, int splits, int64_t stride, int ld, int N,
                                     int K, float* out, int accumulate, int vec) {
  if (vec) {
    const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // 4-column unit
    if (i4 * 4 >= (int64_t)N * K) return;
    const int n = (int)(i4 * 4 / K), k = (int)(i4 * 4 % K);
    const float* base = slab + (int64_t)n * ld + k;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int z = 0;
    for (; z + 16 <= splits; z += 16) {
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const float4*>(base + (int64_t)(z + u) * stride);
#pragma unroll
      for (int u = 0; u < 16; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; z < splits; ++z) {
      const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)z * stride);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out + (int64_t)n * K + k);
    if (accumulate) {
      const float4 a = *o;
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    *o = s;
    return;
  }
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * K) return;
  int n = (int)(i / K), k = (int)(i % K);
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += slab[z * stride + (int64_t)n * ld + k];
  out[i] = accumulate ? out[i] + s : s;
}

// fp32 weights -> padded T copies [rows_p][ld] (8 columns = one 16-B (bf16)
// or two 16-B (fp32) stores per thread) and, for the backward, transposes
// [cols_p][ld_t] through 64x64 LDS tiles (coalesced reads and writes).
template <typename T>
__device__ __forceinline__ void pack_rows(const PackDesc& d) {
  T* dst = (T*)d.dst;
  const int cg = d.ld >> 3;
  const int tot = d.rows_p * cg;
  const bool vec = d.src && d.cols % 4 == 0 && ((uintptr_t)d.src & 15) == 0;
  for (int i = blockIdx.x * NT + threadIdx.x; i < tot; i += gridDim.x * NT) {
    const int r = i / cg, c0 = (i - r * cg) * 8;
    float v[8];
    if (vec && r < d.rows && c0 + 8 <= d.cols) {   // two 16-B loads
      const f32x4* q = reinterpret_cast<const f32x4*>(d.src + (int64_t)r * d.cols + c0);
      const f32x4 a = q[0], b = q[1];
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[k] = a[k]; v[4 + k] = b[k]; }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = c0 + k;
        v[k] = (r < d.rows && c < d.cols) ? d.src[(int64_t)r * d.cols + c] : 0.f;
      }
    }
    T* p = dst + (int64_t)r * d.ld + c0;
    if constexpr (sizeof(T) == 2) {
      bf16x8 h;
#pragma unroll
      for (int k = 0; k < 8; ++k) h[k] = (bf16)v[k];
      *reinterpret_cast<bf16x8*>(p) = h;
    } else {
      *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  }
}

// (d.f32: an fp32 copy -- biases, counters -- in the same launch as T weights)
template <typename T>
__global__ __launch_bounds__(NT) void pack_kernel(PackBatch pb) {
  const PackDesc& d = pb.d[blockIdx.y];
  if (d.f32) pack_rows<float>(d);
  else pack_rows<T>(d);
  if (!d.dst_t) return;
  __shared__ float tile[64][65];
  T* dt = (T*)d.dst_t;
  const int tr = (d.ld_t + 63) / 64, tc = (d.cols_p + 63) / 64;
  for (int t = blockIdx.x; t < tr * tc; t += gridDim.x) {
    const int r0 = (t / tc) * 64, c0 = (t % tc) * 64;
    for (int k = threadIdx.x; k < 64 * 64; k += NT) {
      const int rr = k >> 6, cc = k & 63, r = r0 + rr, c = c0 + cc;
      tile[rr][cc] = (r < d.rows && c < d.cols) ? d.src[(int64_t)r * d.cols + c] : 0.f;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 64 * 64; k += NT) {
      const int cc = k >> 6, rr = k & 63, r = r0 + rr, c = c0 + cc;
      if (c < d.cols_p && r < d.ld_t) St<T>::st(dt + (int64_t)c * d.ld_t + r, tile[rr][cc]);
    }
    __syncthreads();
  }
}

// Column reduction of per-chunk partials part [nchunks][NK][N] (f32) in fp64,
// fused with its consumer.  Grid = (N/64 column groups) x RED_G chunk groups:
// each block sums its chunk range for 64 columns (256 B coalesced rows, 4
// chunk lanes), writes an fp64 block partial to rf.red2 [RED_G][3][N], and the
// last block of each column group (device-scope counter, self-resetting) adds
// the RED_G partials in fixed order and finalises: deterministic, one launch.
// With `shift` (the stats pass's K = t[0]) the shifted sums S0' = sum(t-K),
// S1' = sum((t-K)^2) become S0 = S0' + nK, S1 = S1' + 2K S0' + nK^2.
template <typename T>
__global__ __launch_bounds__(NT) void reduce_fused_kernel(const float* part, int nchunks, int NK,
                                                          int N, int Nr, const T* shift,
                                                          RedFinal rf) {
  __shared__ double red[4 * 3 * 64 + 1];   // one LDS object (the hand-off flag lives in it)
  int* flag = reinterpret_cast<int*>(&red[4 * 3 * 64]);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int cgrp = blockIdx.x, g = blockIdx.y;
  const int n = cgrp * 64 + tx;
  const int per = (nchunks + RED_G - 1) / RED_G;
  const int c0 = g * per, c1 = min(nchunks, c0 + per);
  // stage 1: this block's chunk range, 8 chunk rows x NK loads in flight per
  // lane; out-of-range elements come back as 0 from the buffer descriptor
  // (no per-element branch, which would serialise the loads)
  const __amdgpu_buffer_rsrc_t pr = buf_rsrc(part, (int64_t)nchunks * NK * N * 4);
  constexpr int U = 8;
  double s[3] = {0.0, 0.0, 0.0};
  for (int c = c0 + ty; c < c1; c += 4 * U) {
    float v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = c + 4 * u;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const bool ok = n < N && cc < c1 && k < NK;
        v[u][k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            pr, ok ? ((cc * NK + k) * N + n) * 4 : OOR, 0, 0));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 3; ++k) s[k] += (double)v[u][k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) red[(ty * 3 + k) * 64 + tx] = s[k];
  __syncthreads();
  if (ty == 0 && n < N)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      rf.red2[((int64_t)g * 3 + k) * N + n] =
          ((red[k * 64 + tx] + red[(3 + k) * 64 + tx]) + red[(6 + k) * 64 + tx]) + red[(9 + k) * 64 + tx];
  if (!last_arriver(&rf.counter[cgrp], RED_G, flag)) return;
  // stage 2 (last block of this column group): lane ty sums groups
  // ty*QP .. ty*QP+QP-1 (all loads issued first), then a fixed-order combine
  constexpr int QP = RED_G / 4;
  const __amdgpu_buffer_rsrc_t r2r = buf_rsrc(rf.red2, (int64_t)RED_G * 3 * N * 8);
  {
    double w[QP][3];
#pragma unroll
    for (int q = 0; q < QP; ++q)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const bool ok = n < N && k < NK;
        u32x2 raw = __builtin_amdgcn_raw_buffer_load_b64(
            r2r, ok ? (((ty * QP + q) * 3 + k) * N + n) * 8 : OOR, 0, 0);
        w[q][k] = __builtin_bit_cast(double, raw);
      }
    double t3[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < QP; ++q)
#pragma unroll
      for (int k = 0; k < 3; ++k) t3[k] += w[q][k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 3; ++k) red[(ty * 3 + k) * 64 + tx] = t3[k];
    __syncthreads();
  }
  if (ty != 0 || n >= N) return;
  double v0 = ((red[0 * 64 + tx] + red[3 * 64 + tx]) + red[6 * 64 + tx]) + red[9 * 64 + tx];
  double v1 = ((red[1 * 64 + tx] + red[4 * 64 + tx]) + red[7 * 64 + tx]) + red[10 * 64 + tx];
  double v2 = ((red[2 * 64 + tx] + red[5 * 64 + tx]) + red[8 * 64 + tx]) + red[11 * 64 + tx];
  const bool has_k = shift || rf.shiftf;
  const double K = rf.shiftf ? (double)rf.shiftf[n] : shift ? (double)(float)shift[n] : 0.0;
  red_finalize(rf, n, N, Nr, v0, v1, v2, has_k, K);
}

}  // namespace

namespace {
// Few partial rows (the GEMM epilogues' 64-128): one stage, one launch.
// Block = 32 columns x 8 row groups; each lane sums its rows (all loads in
// flight, fp64, fixed order), the 8 groups are combined in fixed order.
constexpr int SMALL_ROWS = 256;
template <typename T>
__global__ __launch_bounds__(NT) void reduce_small_kernel(const float* part, int nchunks, int NK,
                                                          int N, int Nr, const T* shift,
                                                          RedFinal rf) {
  __shared__ double red[8][3][32];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int n = blockIdx.x * 32 + tx;
  const __amdgpu_buffer_rsrc_t pr = buf_rsrc(part, (int64_t)nchunks * NK * N * 4);
  constexpr int U = SMALL_ROWS / 8;
  double s3[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = ty * U + u;
      const bool ok = n < N && c < nchunks && k < NK;
      v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, ok ? ((c * NK + k) * N + n) * 4 : OOR, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s3[k] += (double)v[u];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) red[ty][k][tx] = s3[k];
  __syncthreads();
  if (ty != 0 || n >= N) return;
  double v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double t = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][k][tx];
    v[k] = t;
  }
  const bool has_k = shift || rf.shiftf;
  const double K = rf.shiftf ? (double)rf.shiftf[n] : shift ? (double)(float)shift[n] : 0.0;
  red_finalize(rf, n, N, Nr, v[0], v[1], v[2], has_k, K);
}
}  // namespace

dcnr_status reduce_fused(int precision, const float* part, int nchunks, int NK, int N, int Nr,
                         const void* shift, const RedFinal& rf, hipStream_t s) {
  if (N <= 0 || N > 64 * RED_MAX_CGRP || NK < 1 || NK > 3) {
    set_error("reduce: unsupported width %d / components %d", N, NK);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (nchunks <= SMALL_ROWS) {
    const dim3 g((unsigned)cdiv(N, 32));
    if (precision == DCNR_PREC_BF16)
      hipLaunchKernelGGL(reduce_small_kernel<bf16>, g, dim3(NT), 0, s, part, nchunks, NK, N, Nr,
                         (const bf16*)shift, rf);
    else
      hipLaunchKernelGGL(reduce_small_kernel<float>, g, dim3(NT), 0, s, part, nchunks, NK, N, Nr,
                         (const float*)shift, rf);
    DCNR_LAUNCH_CHECK();
    return DCNR_OK;
  }
  dim3 grid((unsigned)cdiv(N, 64), RED_G);
  if (precision == DCNR_PREC_BF16)
    hipLaunchKernelGGL(reduce_fused_kernel<bf16>, grid, dim3(NT), 0, s, part, nchunks, NK, N, Nr,
                       (const bf16*)shift, rf);
  else
    hipLaunchKernelGGL(reduce_fused_kernel<float>, grid, dim3(NT), 0, s, part, nchunks, NK, N, Nr,
                       (const float*)shift, rf);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

// ================================================================== API
dcnr_status pack_weights(int precision, const PackBatch& pb, hipStream_t s) {
  if (pb.n == 0) return DCNR_OK;
  for (int i = 0; i < pb.n; ++i)
    if (pb.d[i].ld % 8) {
      set_error("pack: leading dimension %d not a multiple of 8", pb.d[i].ld);
      return DCNR_UNSUPPORTED_SHAPE;
    }
  // one 8-column group per thread for a 512 x 512 matrix (the transposes'
  // 64 x 64 tiles need 64 blocks)
  int gx = 64;
  for (int i = 0; i < pb.n; ++i)
    gx = std::max<int>(gx, (int)std::min<int64_t>(256, cdiv((int64_t)pb.d[i].rows_p * (pb.d[i].ld >> 3), NT)));
  dim3 grid(gx, pb.n);
  if (precision == DCNR_PREC_BF16) hipLaunchKernelGGL(pack_kernel<bf16>, grid, dim3(NT), 0, s, pb);
  else hipLaunchKernelGGL(pack_kernel<float>, grid, dim3(NT), 0, s, pb);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

template <typename T>
static dcnr_status col_stats_impl(const void* t, int64_t B, int N, int ld, float* part, int* nc,
                                  hipStream_t s) {
  StatsOp<T> op{(const T*)t, ld};
  return run_rowcol<T, 2>(op, B, N, part, nc, s);
}
dcnr_status col_stats(int precision, const void* t, int64_t B, int N, int ld, float* part,
                      int* nchunks, hipStream_t s) {
  return precision == DCNR_PREC_BF16 ? col_stats_impl<bf16>(t, B, N, ld, part, nchunks, s)
                                     : col_stats_impl<float>(t, B, N, ld, part, nchunks, s);
}

template <typename T>
static dcnr_status col_sum_impl(const void* x, int64_t B, int N, int ld, float* part, int* nc,
                                hipStream_t s) {
  ColSumOp<T> op{(const T*)x, ld};
  return run_rowcol<T, 1>(op, B, N, part, nc, s);
}
dcnr_status col_sum(int precision, const void* x, int64_t B, int N, int ld, float* part,
                    int* nchunks, hipStream_t s) {
  return precision == DCNR_PREC_BF16 ? col_sum_impl<bf16>(x, B, N, ld, part, nchunks, s)
                                     : col_sum_impl<float>(x, B, N, ld, part, nchunks, s);
}

// eval-mode finalize of several BN layers in one launch (blockIdx.y = layer):
// the same per-column arithmetic as bn_finalize_kernel's running-stat branch
__global__ void bn_eval_multi_kernel(BnEvalBatch b) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const BnFinal& f = b.f[blockIdx.y];
  if (n >= b.N) return;
  if (n >= b.Nr) {
    f.scale[n] = 0.f; f.shift[n] = 0.f; f.mean[n] = 0.f; f.invstd[n] = 0.f;
    return;
  }
  const double mean = f.rmean[n], var = f.rvar[n];
  float inv = (float)(1.0 / sqrt(var + (double)BN_EPS));
  float sc = f.gamma[n] * inv;
  f.scale[n] = sc;
  f.shift[n] = f.beta[n] - (float)mean * sc;
  f.mean[n] = (float)mean;
  f.invstd[n] = inv;
}

dcnr_status bn_eval_finalize(const BnEvalBatch& b, hipStream_t s) {
  if (b.n <= 0) return DCNR_OK;
  hipLaunchKernelGGL(bn_eval_multi_kernel, dim3((unsigned)cdiv(b.N, NT), (unsigned)b.n), dim3(NT), 0, s, b);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status bn_finalize2(const double* sums, int N, int Nr, int train, const BnFinal& f,
                         hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)cdiv(N, NT)), dim3(NT), 0, s, sums, N, Nr,
                     train, f);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status bn_bwd_coef(const double* sums, int N, int Nr, const float* gamma, const float* invstd,
                        float* coef, int train, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((unsigned)cdiv(N, NT)), dim3(NT), 0, s, sums, N, Nr,
                     gamma, invstd, coef, train);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}


template <typename T>
static dcnr_status bn_relu_drop_impl(const void* t, void* a, int64_t B, int N, int ld,
                                     const float* sc, const float* sh, float p, uint64_t seed,
                                     int layer, hipStream_t s, uint8_t* bits) {
  BnReluDropOp<T> op{(const T*)t, (T*)a, ld, sc, sh, p > 0.f ? 1.f / (1.f - p) : 1.f,
                     drop_thresh16(p), seed, layer, p > 0.f, bits};
  return run_rowcol<T, 0>(op, B, N, nullptr, nullptr, s);
}
dcnr_status bn_relu_drop(int precision, const void* t, void* a, int64_t B, int N, int ld,
                         const float* scale, const float* shift, float p, uint64_t seed,
                         int layer, hipStream_t s, uint8_t* bits) {
  return precision == DCNR_PREC_BF16
             ? bn_relu_drop_impl<bf16>(t, a, B, N, ld, scale, shift, p, seed, layer, s, bits)
             : bn_relu_drop_impl<float>(t, a, B, N, ld, scale, shift, p, seed, layer, s, nullptr);
}

template <typename T>
static dcnr_status bn_add_relu_impl(const void* t, const void* x, void* out, int64_t B, int N,
                                    int ld, const float* sc, const float* sh, hipStream_t s,
                                    uint8_t* bits) {
  BnAddReluOp<T> op{(const T*)t, (const T*)x, (T*)out, ld, sc, sh, bits};
  return run_rowcol<T, 0>(op, B, N, nullptr, nullptr, s);
}
dcnr_status bn_add_relu2(int precision, const void* t, const void* x, void* out, int64_t B, int N,
                         int ld, const float* scale, const float* shift, hipStream_t s,
                         uint8_t* bits) {
  return precision == DCNR_PREC_BF16
             ? bn_add_relu_impl<bf16>(t, x, out, B, N, ld, scale, shift, s, bits)
             : bn_add_relu_impl<float>(t, x, out, B, N, ld, scale, shift, s, nullptr);
}

template <typename T>
static dcnr_status bn_add_relu_head_impl(const void* t, const void* x, void* out, int64_t B, int N,
                                         int ld, const float* sc, const float* sh, const float* wf,
                                         int Nr, const float* zc, const float* bf, float* logits,
                                         uint8_t* bits, hipStream_t s) {
  BnAddReluHeadOp<T> op{(const T*)t, (const T*)x, (T*)out, ld, sc, sh, wf, Nr, zc, bf, logits, bits};
  return run_rowcol<T, 0>(op, B, N, nullptr, nullptr, s);
}
bool bn_add_relu_head_supported(int precision, int N) {
  return N / (precision == DCNR_PREC_BF16 ? 8 : 4) == 64;
}
dcnr_status bn_add_relu_head(int precision, const void* t, const void* x, void* out, int64_t B,
                             int N, int ld, const float* scale, const float* shift,
                             const float* wf, int Nr, const float* zc, const float* bf,
                             float* logits, hipStream_t s, uint8_t* bits) {
  if (!bn_add_relu_head_supported(precision, N)) {
    set_error("bn_add_relu_head: needs a wave per row (N=%d)", N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  return precision == DCNR_PREC_BF16
             ? bn_add_relu_head_impl<bf16>(t, x, out, B, N, ld, scale, shift, wf, Nr, zc, bf, logits, bits, s)
             : bn_add_relu_head_impl<float>(t, x, out, B, N, ld, scale, shift, wf, Nr, zc, bf, logits, nullptr, s);
}

template <typename T>
static dcnr_status bwd2_stats_impl(const void* G, const float* dz, const float* wf, const void* out,
                                   const void* t, const float* mean, const float* invstd,
                                   int64_t B, int N, int ld, void* du, float* part, int* nc,
                                   hipStream_t s, const void* x, const float* sc, const float* sh) {
  if (!G && x) {
    Bwd2StatsOp<T, false, true> op{nullptr, dz, wf, (const T*)x, (const T*)t, mean, invstd, ld,
                                   (T*)du, sc, sh};
    return run_rowcol<T, 3>(op, B, N, part, nc, s);
  }
  if (G) {
    Bwd2StatsOp<T, true> op{(const T*)G, dz, wf, (const T*)out, (const T*)t, mean, invstd, ld,
                            (T*)du};
    return run_rowcol<T, 3>(op, B, N, part, nc, s);
  }
  Bwd2StatsOp<T, false> op{(const T*)G, dz, wf, (const T*)out, (const T*)t, mean, invstd, ld,
                           (T*)du};
  return run_rowcol<T, 3>(op, B, N, part, nc, s);
}
dcnr_status bwd_bn2_stats3(int precision, const void* G, const float* dz, const float* wf,
                           const void* out, const void* t, const float* mean, const float* invstd,
                           int64_t B, int N, int ld, void* du, float* part, int* nchunks,
                           hipStream_t s, const void* x, const float* sc, const float* sh) {
  return precision == DCNR_PREC_BF16
             ? bwd2_stats_impl<bf16>(G, dz, wf, out, t, mean, invstd, B, N, ld, du, part, nchunks, s, x, sc, sh)
             : bwd2_stats_impl<float>(G, dz, wf, out, t, mean, invstd, B, N, ld, du, part, nchunks, s, x, sc, sh);
}

template <typename T>
static dcnr_status bwd2_apply_impl(const void* du, const void* t, const float* mean,
                                   const float* invstd, const float* coef, int64_t B, int N,
                                   int ld, void* dt, float* part, int* nc, hipStream_t s) {
  Bwd2ApplyOp<T> op{(const T*)du, (const T*)t, mean, invstd, coef, ld, N, (T*)dt};
  return run_rowcol<T, 0>(op, B, N, nullptr, nullptr, s);
}
dcnr_status bwd_bn2_apply_rank1(const uint8_t* bits, const float* dz, const float* wf, const void* t,
                                const float* mean, const float* invstd, const float* coef,
                                int64_t B, int N, int ld, void* dt, hipStream_t s) {
  Bwd2ApplyRank1Op<bf16> op{bits, dz, wf, (const bf16*)t, mean, invstd, coef, ld, N, (bf16*)dt};
  return run_rowcol<bf16, 0>(op, B, N, nullptr, nullptr, s);
}
dcnr_status bwd_bn2_apply2(int precision, const void* du, const void* t, const float* mean,
                           const float* invstd, const float* coef, int64_t B, int N, int ld,
                           void* dt, float* part, int* nchunks, hipStream_t s) {
  return precision == DCNR_PREC_BF16
             ? bwd2_apply_impl<bf16>(du, t, mean, invstd, coef, B, N, ld, dt, part, nchunks, s)
             : bwd2_apply_impl<float>(du, t, mean, invstd, coef, B, N, ld, dt, part, nchunks, s);
}

template <typename T>
static dcnr_status bwd1_stats_impl(void* da, const void* t, const float* sc, const float* sh,
                                   const float* mean, const float* invstd, int64_t B, int N,
                                   int ld, float p, uint64_t seed, int layer, float* part, int* nc,
                                   hipStream_t s) {
  Bwd1StatsOp<T> op{(T*)da, (const T*)t, sc, sh, mean, invstd, ld,
                    p > 0.f ? 1.f / (1.f - p) : 1.f, drop_thresh16(p), seed, layer, p > 0.f};
  return run_rowcol<T, 2>(op, B, N, part, nc, s);
}
dcnr_status bwd_bn1_stats(int precision, void* da_dr, const void* t, const float* scale,
                          const float* shift, const float* mean, const float* invstd, int64_t B,
                          int N, int ld, float p, uint64_t seed, int layer, float* part,
                          int* nchunks, hipStream_t s) {
  return precision == DCNR_PREC_BF16
             ? bwd1_stats_impl<bf16>(da_dr, t, scale, shift, mean, invstd, B, N, ld, p, seed,
                                     layer, part, nchunks, s)
             : bwd1_stats_impl<float>(da_dr, t, scale, shift, mean, invstd, B, N, ld, p, seed,
                                      layer, part, nchunks, s);
}

template <typename T>
static dcnr_status bwd1_apply_impl(const void* dr, const void* t, const float* mean,
                                   const float* invstd, const float* coef, int64_t B, int N,
                                   int ld, void* dt, float* part, int* nc, hipStream_t s) {
  Bwd1ApplyOp<T> op{(const T*)dr, (const T*)t, mean, invstd, coef, ld, N, (T*)dt};
  return run_rowcol<T, 0>(op, B, N, nullptr, nullptr, s);
}
dcnr_status bwd_bn1_apply2(int precision, const void* dr, const void* t, const float* mean,
                           const float* invstd, const float* coef, int64_t B, int N, int ld,
                           void* dt, float* part, int* nchunks, hipStream_t s) {
  return precision == DCNR_PREC_BF16
             ? bwd1_apply_impl<bf16>(dr, t, mean, invstd, coef, B, N, ld, dt, part, nchunks, s)
             : bwd1_apply_impl<float>(dr, t, mean, invstd, coef, B, N, ld, dt, part, nchunks, s);
}

dcnr_status sums_to_grad(const double* sums, int N, float* out, int accumulate, hipStream_t s) {
  if (N <= 0) return DCNR_OK;
  hipLaunchKernelGGL(sums_to_grad_kernel, dim3((unsigned)cdiv(N, NT)), dim3(NT), 0, s, sums, N,
                     out, accumulate);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status splitk_reduce(const float* slab, int splits, int64_t slab_stride, int ld_slab, int N,
                          int K, float* out, int accumulate, hipStream_t s) {
  int64_t tot = (int64_t)N * K;
  if (tot <= 0) return DCNR_OK;
  const int vec = K % 4 == 0 && ld_slab % 4 == 0 && slab_stride % 4 == 0 &&
                  (uintptr_t)slab % 16 == 0 && (uintptr_t)out % 16 == 0;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)cdiv(vec ? tot / 4 : tot, NT)), dim3(NT),
                     0, s, slab, splits, slab_stride, ld_slab, N, K, out, accumulate, vec);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

namespace {
// out[n][k] (+)= sum_z slab[z][k][n]: the weight-gradient GEMM's transposed
// slabs (gemm_dw.hip stores 4 consecutive n per lane as one 16-B store).  A
// block takes 64 k x 16 n: reads along n (4 lanes x 16 B per 64-B row
// segment, 16 slab loads in flight per lane), sums in fixed z order (the same
// bits as summing the untransposed slabs), transposes through LDS, writes
// rows of out along k (16-B stores when out's rows allow).
// (Several thread groups per output tile, each summing a contiguous share of
// the splits, measured 12-13 us alone either way per 512 x 512 call and
// 40-54 us under the concurrent dX chain; one group kept -- the summation
// order of the earlier rounds.)
__global__ __launch_bounds__(256) void splitk_reduce_t_kernel(const float* slab, int splits,
                                                              int64_t stride, int ld, int N, int K,
                                                              float* out, int accumulate, int vec_out) {
  __shared__ float t[RT_K][RT_N + 1];
  splitk_t_sum(slab, splits, stride, ld, N, K, blockIdx.x, blockIdx.y, threadIdx.x, t);
  __syncthreads();
  splitk_t_store(N, K, out, accumulate, vec_out, blockIdx.x, blockIdx.y, threadIdx.x, t);
}
}  // namespace

dcnr_status splitk_reduce_t(const float* slab, int splits, int64_t slab_stride, int ld_slab, int N,
                            int K, float* out, int accumulate, hipStream_t s) {
  if ((int64_t)N * K <= 0) return DCNR_OK;
  if (ld_slab % 4 || slab_stride % 4 || (uintptr_t)slab % 16) {
    set_error("splitk_reduce_t: slab not 16-B aligned");
    return DCNR_UNSUPPORTED_SHAPE;
  }
  const int vec_out = K % 4 == 0 && (uintptr_t)out % 16 == 0;
  hipLaunchKernelGGL(splitk_reduce_t_kernel, dim3((unsigned)cdiv(K, RT_K), (unsigned)cdiv(N, RT_N)),
                     dim3(256), 0, s, slab, splits, slab_stride, ld_slab, N, K, out, accumulate,
                     vec_out);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

namespace {
// a few words: one wave (the runtime's fill blit measured 5.7 us per step on
// the 4-B error word, profiles/r03at_step_timeline.txt)
__global__ __launch_bounds__(64) void zero_words_kernel(int* p, int n) {
  for (int i = threadIdx.x; i < n; i += 64) p[i] = 0;
}
__global__ __launch_bounds__(64) void mirror_word_kernel(const int* src, int* dst) {
  // dst may be pinned host memory: a system-scope store, visible to the host
  // once the stream's work up to here has completed
  if (threadIdx.x == 0) __hip_atomic_store(dst, *src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

dcnr_status fill_zero(void* p, size_t bytes, hipStream_t s) {
  if (!bytes) return DCNR_OK;
  if (bytes <= 4096 && !(bytes & 3) && !((uintptr_t)p & 3)) {
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, s, (int*)p, (int)(bytes / 4));
    DCNR_LAUNCH_CHECK();
    return DCNR_OK;
  }
  DCNR_HIP(hipMemsetAsync(p, 0, bytes, s));
  return DCNR_OK;
}

dcnr_status mirror_word(const int* src, int* dst, hipStream_t s) {
  hipLaunchKernelGGL(mirror_word_kernel, dim3(1), dim3(64), 0, s, src, dst);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

namespace {
constexpr int ZB_MAX = 66;
constexpr int ZB_CHUNK = NT * 16;   // 16-B units per block
struct ZeroBatch {
  char* p[ZB_MAX]; int64_t bytes[ZB_MAX]; int64_t blk0[ZB_MAX + 1]; int n;
};
// zero n buffers in one launch: 16-B stores for the body, 4-B for a tail
__global__ __launch_bounds__(NT) void zero_multi_kernel(ZeroBatch zb) {
  int t = 0;
  while (t + 1 < zb.n && (int64_t)blockIdx.x >= zb.blk0[t + 1]) ++t;
  char* p = zb.p[t];
  const int64_t n16 = zb.bytes[t] / 16;
  const int64_t u0 = ((int64_t)blockIdx.x - zb.blk0[t]) * ZB_CHUNK;
  for (int64_t u = u0 + threadIdx.x; u < min(n16, u0 + ZB_CHUNK); u += NT)
    reinterpret_cast<uint4*>(p)[u] = make_uint4(0, 0, 0, 0);
  if ((int64_t)blockIdx.x == zb.blk0[t + 1] - 1)
    for (int64_t i = n16 * 16 + threadIdx.x * 4; i < zb.bytes[t]; i += NT * 4)
      *reinterpret_cast<float*>(p + i) = 0.f;
}
}  // namespace

dcnr_status fill_zero_multi(int n, void* const* ptrs, const int64_t* bytes, hipStream_t s) {
  for (int o = 0; o < n; o += ZB_MAX) {
    ZeroBatch zb;
    zb.n = std::min(ZB_MAX, n - o);
    zb.blk0[0] = 0;
    for (int i = 0; i < zb.n; ++i) {
      zb.p[i] = (char*)ptrs[o + i];
      zb.bytes[i] = bytes[o + i];
      zb.blk0[i + 1] = zb.blk0[i] + std::max<int64_t>(1, cdiv(bytes[o + i] / 16, ZB_CHUNK));
    }
    bool aligned = true;
    for (int i = 0; i < zb.n; ++i)
      aligned = aligned && !((uintptr_t)zb.p[i] & 15) && !(zb.bytes[i] & 3);
    if (!aligned) {   // unaligned buffers (not from torch's allocator): plain memsets
      for (int i = 0; i < zb.n; ++i) {
        dcnr_status st = fill_zero(zb.p[i], (size_t)zb.bytes[i], s);
        if (st != DCNR_OK) return st;
      }
      continue;
    }
    hipLaunchKernelGGL(zero_multi_kernel, dim3((unsigned)zb.blk0[zb.n]), dim3(NT), 0, s, zb);
    DCNR_LAUNCH_CHECK();
  }
  return DCNR_OK;
}

}  // namespace dcnr
