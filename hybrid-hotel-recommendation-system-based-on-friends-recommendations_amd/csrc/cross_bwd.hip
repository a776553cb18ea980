// Backward of the cross network (CrossLayer, reference train.py:88-99,
// x_{l+1} = x_l + x_l (x_l . w_l) + b_l, and the cross half of
// final_linear, train.py:166-170), in low-rank form.
//
// Every forward state is x_l = a_l x_0 + sum_{j<l} e_lj b_j and every
// backward gradient g_l = dL/dx_l is f_l w_f + sum_m c_lm w_m (g_L = dz w_f;
// g_l = (1 + s_l) g_{l+1} + (g_{l+1} . x_l) w_l), with per-sample scalars
// built from s_l = x_l . w_l, u_m = x_0 . w_m, u_f = x_0 . w_f (saved by the
// train forward, GcOut::sc) and the constant Gram terms b_j . w_m, b_j . w_f.
// So the backward never touches a D-vector per sample:
//
//   cross_coef_kernel   per sample: dx0_cross coefficients (c_0m, f_0) -> coef
//                       [B][L+1], the x_0 weights of dw_l and dw_f -> alpha
//                       [B][L+1], and the batch sums of the remaining scalar
//                       coefficients (block partials, fixed-order reduction)
//   x0_alpha_kernel     sum_b alpha_k(b) x_0[b] over the saved x0 (one read of
//   (+ _reduce)         the [B][Dp] x0 the deep tower already stores; in bf16
//                       mode that is the bf16 x0, so dw_l and dw_f[H:] see x_0
//                       rounded to bf16 like the deep tower's W0 gradient)
//   cross_final_kernel  dw_l = X0a_l + sum_j beta_lj b_j,
//                       dw_f[H:] = X0a_L + sum_j betaf_j b_j,
//                       db_l = gam_lf w_f + sum_m gam_lm w_m, db_f = sum dz
//
// and the embedding backward (embed_bwd.hip) adds sum_k coef_k V_k (V =
// w_0..w_{L-1}, w_f) to the deep part of each embedding row's sum.  This
// replaced a kernel that re-gathered every x0 row (235 MB), read the deep
// dx0 (239 MB) and wrote the total dx0 (235 MB): ~200 us -> ~25 us at the
// bench size.  All reductions are in fixed order (deterministic).
#include "dcnr_internal.h"

#include <algorithm>
#include <cstring>

namespace dcnr {
namespace {

constexpr int CT = 256;          // threads per block
constexpr int XA_ROWS = 256;     // x0 rows per x0_alpha_kernel block
constexpr int XA_W = 8;          // its waves
constexpr int XA_T = XA_W * WAVE;

// scalar slots reduced over the batch:
//   gam[l][v]  l < L, v <= L  (db_l coefficient on w_v, v == L: w_f)
//   bet[l][j]  l < L, j < L   (dw_l coefficient on b_j)
//   betf[j]    j < L          (dw_f coefficient on b_j)
//   dbf
__host__ __device__ constexpr int ns_of(int L) { return 2 * L * L + 2 * L + 1; }

// gram[j * (L + 1) + v] = b_j . V_v  (V_v = w_v, V_L = w_f[H:]); one wave per pair
__global__ __launch_bounds__(WAVE) void cross_gram_kernel(CrossParams cp, int D, float* gram) {
  const int L = cp.L, lane = threadIdx.x & 63;
  {
    const int p = blockIdx.x;
    const int j = p / (L + 1), v = p % (L + 1);
    const float* a = cp.b[j];
    const float* bv = v < L ? cp.w[v] : cp.wf_cross;
    float d = 0.f;
    for (int e = lane; e < D; e += WAVE) d += a[e] * bv[e];
    d = wave_sum_dpp(d);
    if (lane == 0) gram[p] = d;
  }
}

template <int L>
__global__ __launch_bounds__(CT) void cross_coef_kernel(const float* sc, const float* dz,
                                                        const float* gram, int64_t B,
                                                        float* coef, float* alpha, float* part) {
  constexpr int NS = ns_of(L), V = L + 1, LL = L > 0 ? L : 1;
  __shared__ float red[CT / WAVE][NS];
  const int64_t b = (int64_t)blockIdx.x * CT + threadIdx.x;
  const bool valid = b < B;
  const int64_t bc = valid ? b : 0;
  float s[LL], u[V], G[LL][V];
#pragma unroll
  for (int l = 0; l < L; ++l) s[l] = sc[bc * (2 * L + 1) + l];
#pragma unroll
  for (int v = 0; v < V; ++v) u[v] = sc[bc * (2 * L + 1) + L + v];
#pragma unroll
  for (int j = 0; j < L; ++j)
#pragma unroll
    for (int v = 0; v < V; ++v) G[j][v] = gram[j * V + v];
  const float dzb = valid ? dz[b] : 0.f;
  // forward coefficients: x_l = xa[l] x_0 + sum_j xe[l][j] b_j
  float xa[L + 1], xe[L + 1][LL];
  xa[0] = 1.f;
#pragma unroll
  for (int j = 0; j < L; ++j) xe[0][j] = 0.f;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float m = 1.f + s[l];
    xa[l + 1] = m * xa[l];
#pragma unroll
    for (int j = 0; j < L; ++j) xe[l + 1][j] = j == l ? 1.f : m * xe[l][j];
  }
  float acc[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] = 0.f;
  float* gam = acc;                       // [L][V]
  float* bet = acc + L * V;               // [L][L]
  float* betf = acc + L * V + L * L;      // [L]
  // dw_f[H:] = sum_b dz x_L
  const float af = dzb * xa[L];
#pragma unroll
  for (int j = 0; j < L; ++j) betf[j] = dzb * xe[L][j];
  acc[NS - 1] = dzb;
  // g = sum_v gc[v] V_v, g_L = dz w_f
  float gc[V];
#pragma unroll
  for (int v = 0; v < L; ++v) gc[v] = 0.f;
  gc[L] = dzb;
  float al[LL];
#pragma unroll
  for (int l = L - 1; l >= 0; --l) {
    // gx = g_{l+1} . x_l
    float gx = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float xv = xa[l] * u[v];
#pragma unroll
      for (int j = 0; j < L; ++j) xv += xe[l][j] * G[j][v];
      gx += gc[v] * xv;
    }
#pragma unroll
    for (int v = 0; v < V; ++v) gam[l * V + v] = gc[v];   // db_l += g_{l+1}
    al[l] = gx * xa[l];                                    // dw_l += gx x_l
#pragma unroll
    for (int j = 0; j < L; ++j) bet[l * L + j] = gx * xe[l][j];
    const float m = 1.f + s[l];
#pragma unroll
    for (int v = 0; v < V; ++v) gc[v] *= m;
    gc[l] += gx;
  }
  if (valid) {
#pragma unroll
    for (int v = 0; v < V; ++v) coef[b * V + v] = gc[v];
#pragma unroll
    for (int l = 0; l < L; ++l) alpha[b * V + l] = al[l];
    alpha[b * V + L] = af;
  }
  // block partials of the NS batch sums: wave trees, then waves in order
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const float t = wave_sum_dpp(acc[i]);
    if (lane == 0) red[w][i] = t;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NS; i += CT) {
    float t = red[0][i];
    for (int ww = 1; ww < CT / WAVE; ++ww) t += red[ww][i];
    part[(int64_t)blockIdx.x * NS + i] = t;
  }
}

// scal[i] = sum over blocks of part[blk][i]: thread t takes blocks t, t+CT, ...
// in order, then a fixed LDS tree
__global__ __launch_bounds__(CT) void cross_scalar_reduce_kernel(const float* part, int nblk,
                                                                 int NS, float* scal) {
  __shared__ float red[CT];
  const int i = blockIdx.x;
  float t = 0.f;
  for (int k = threadIdx.x; k < nblk; k += CT) t += part[(int64_t)k * NS + i];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int o = CT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) scal[i] = red[0];
}

// part[blk][k][c] = sum over this block's XA_ROWS rows b of alpha[b][k] * x0[b][c].
// Wave w takes rows w*RW .. w*RW+RW-1 of the block (8 in flight), lane L the
// 8 columns 8L..8L+7 (one 16-B bf16 / two 16-B fp32 loads per row), 512
// columns per pass; the waves' sums are added in wave order through LDS.
template <typename T, int V>
__global__ __launch_bounds__(XA_T) void x0_alpha_kernel(const T* x0, int ldx, int D,
                                                        const float* alpha, int64_t B,
                                                        float* part) {
  constexpr int KM = V, RW = XA_ROWS / XA_W, U = 8;
  __shared__ float red[KM][8 * WAVE];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r0 = (int64_t)blockIdx.x * XA_ROWS + (int64_t)w * RW;
  const int64_t r1 = std::min<int64_t>(B, r0 + RW);
  static_assert(RW <= WAVE, "one alpha row per lane");
  // lane j holds alpha of row r0 + j; rows are broadcast with readlane
  float al[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) al[k] = (k < V && r0 + lane < r1) ? alpha[(r0 + lane) * V + k] : 0.f;
  for (int c0 = 0; c0 < D; c0 += 8 * WAVE) {
    const int c = c0 + 8 * lane;
    const bool on = c < ldx;
    float acc[KM][8];
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[k][i] = 0.f;
    for (int64_t b = r0; b < r1; b += U) {
      float xv[U][8];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const bool ok = on && b + q < r1;
        if constexpr (sizeof(T) == 2) {
          bf16x8 h = ok ? *reinterpret_cast<const bf16x8*>(x0 + (b + q) * ldx + c) : bf16x8{};
#pragma unroll
          for (int i = 0; i < 8; ++i) xv[q][i] = (float)h[i];
        } else {
          f32x4 lo = ok ? *reinterpret_cast<const f32x4*>(x0 + (b + q) * ldx + c) : f32x4{};
          f32x4 hi = ok ? *reinterpret_cast<const f32x4*>(x0 + (b + q) * ldx + c + 4) : f32x4{};
#pragma unroll
          for (int i = 0; i < 4; ++i) { xv[q][i] = lo[i]; xv[q][4 + i] = hi[i]; }
        }
      }
#pragma unroll
      for (int q = 0; q < U; ++q)
        if (b + q < r1)
#pragma unroll
          for (int k = 0; k < KM; ++k)
            if (k < V) {
              const float a = __int_as_float(
                  __builtin_amdgcn_readlane(__float_as_int(al[k]), (int)(b + q - r0)));
#pragma unroll
              for (int i = 0; i < 8; ++i) acc[k][i] += a * xv[q][i];
            }
    }
    for (int ww = 0; ww < XA_W; ++ww) {   // waves added in order
      if (w == ww)
#pragma unroll
        for (int k = 0; k < KM; ++k)
#pragma unroll
          for (int i = 0; i < 8; ++i)
            red[k][8 * lane + i] = (ww ? red[k][8 * lane + i] : 0.f) + acc[k][i];
      __syncthreads();
    }
    for (int i = threadIdx.x; i < V * 8 * WAVE; i += XA_T) {
      const int k = i / (8 * WAVE), cc = i % (8 * WAVE);
      if (c0 + cc < D) part[((int64_t)blockIdx.x * V + k) * D + c0 + cc] = red[k][cc];
    }
    __syncthreads();
  }
}

// X0a[k][c] = sum over blocks q of part[q][k][c]: block = 64 (k, c) slots x
// RG block groups (group g sums q = g, g + RG, ... in order; groups added in
// order)
constexpr int RG = 16;
__global__ __launch_bounds__(64 * RG) void x0_alpha_reduce_kernel(const float* part, int nx,
                                                                  int VD, float* x0a) {
  __shared__ float red[RG][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + tx;
  constexpr int U = 8;
  float t = 0.f;
  for (int q = ty; q < nx; q += RG * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = (i < VD && q + RG * u < nx) ? part[(int64_t)(q + RG * u) * VD + i] : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) t += v[u];
  }
  red[ty][tx] = t;
  __syncthreads();
  if (ty == 0 && i < VD) {
    float r = red[0][tx];
    for (int g = 1; g < RG; ++g) r += red[g][tx];
    x0a[i] = r;
  }
}

struct FinalArgs {
  CrossParams cp;
  float* dw[8]; float* db[8]; float* dwf; float* dbf;
  int D, L, accumulate;
};

// one thread per element e < D: every cross-gradient vector's element e
__global__ __launch_bounds__(CT) void cross_final_kernel(FinalArgs a, const float* x0a_,
                                                         const float* scal) {
  const int e = blockIdx.x * CT + threadIdx.x;
  const int L = a.L, V = L + 1, D = a.D;
  const float* gam = scal;
  const float* bet = scal + L * V;
  const float* betf = scal + L * V + L * L;
  if (e == 0) *a.dbf = a.accumulate ? *a.dbf + scal[ns_of(L) - 1] : scal[ns_of(L) - 1];
  if (e >= D) return;
  float x0a[8];
  for (int k = 0; k < V; ++k) x0a[k] = x0a_[k * D + e];
  float bj[8];
  for (int j = 0; j < L; ++j) bj[j] = a.cp.b[j][e];
  for (int l = 0; l < L; ++l) {
    float dw = x0a[l];
    for (int j = 0; j < L; ++j) dw += bet[l * L + j] * bj[j];
    float db = gam[l * V + L] * a.cp.wf_cross[e];
    for (int m = 0; m < L; ++m) db += gam[l * V + m] * a.cp.w[m][e];
    a.dw[l][e] = a.accumulate ? a.dw[l][e] + dw : dw;
    a.db[l][e] = a.accumulate ? a.db[l][e] + db : db;
  }
  float dwf = x0a[L];
  for (int j = 0; j < L; ++j) dwf += betf[j] * bj[j];
  a.dwf[e] = a.accumulate ? a.dwf[e] + dwf : dwf;
}

}  // namespace

size_t cross_bwd_scratch_bytes(int D, int L, int64_t B) {
  const int V = L + 1;
  const int64_t nblk = cdiv(B, CT), nx = cdiv(B, XA_ROWS);
  return (size_t)(64 + nblk * ns_of(L) + ns_of(L) + nx * V * D + V * D) * 4 + 1024;
}

dcnr_status cross_backward(const CrossParams& cp, int D, const float* sc, const float* dz,
                           const void* x0, int x0_bf16, int ldx, int64_t B, const CrossGrads& gr,
                           float* coef, float* alpha, void* scratch, size_t scratch_bytes,
                           int accumulate, hipStream_t s) {
  const int L = cp.L, V = L + 1, NS = ns_of(L);
  if (L < 0 || L > 7) {
    set_error("cross backward: n_cross_layers=%d unsupported (0..7)", L);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (B <= 0) return DCNR_OK;
  if (scratch_bytes < cross_bwd_scratch_bytes(D, L, B)) {
    set_error("cross backward: scratch too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  const int nblk = (int)cdiv(B, CT), nx = (int)cdiv(B, XA_ROWS);
  float* gram = (float*)scratch;             // [64]
  float* part = gram + 64;                   // [nblk][NS]
  float* scal = part + (int64_t)nblk * NS;   // [NS]
  float* xpart = scal + NS;                  // [nx][V][D]
  float* x0a = xpart + (int64_t)nx * V * D;   // [V][D]
  if (L > 0) {
    hipLaunchKernelGGL(cross_gram_kernel, dim3((unsigned)(L * (L + 1))), dim3(WAVE), 0, s, cp, D,
                       gram);
    DCNR_LAUNCH_CHECK();
  }
  switch (L) {
#define CASE(n)                                                                              \
  case n:                                                                                    \
    hipLaunchKernelGGL(cross_coef_kernel<n>, dim3((unsigned)nblk), dim3(CT), 0, s, sc, dz,   \
                       gram, B, coef, alpha, part);                                          \
    break;
    CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7)
#undef CASE
  }
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(cross_scalar_reduce_kernel, dim3((unsigned)NS), dim3(CT), 0, s, part, nblk,
                     NS, scal);
  DCNR_LAUNCH_CHECK();
  if (ldx % 8 || ((uintptr_t)x0 & 15)) {
    set_error("cross backward: x0 rows must be 16-B aligned (ld %d)", ldx);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  switch (V) {
#define CASE(v)                                                                           \
  case v:                                                                                 \
    if (x0_bf16)                                                                          \
      hipLaunchKernelGGL((x0_alpha_kernel<bf16, v>), dim3((unsigned)nx), dim3(XA_T), 0, s, \
                         (const bf16*)x0, ldx, D, alpha, B, xpart);                        \
    else                                                                                  \
      hipLaunchKernelGGL((x0_alpha_kernel<float, v>), dim3((unsigned)nx), dim3(XA_T), 0, s, \
                         (const float*)x0, ldx, D, alpha, B, xpart);                       \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
  }
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(x0_alpha_reduce_kernel, dim3((unsigned)cdiv(V * D, 64)), dim3(64 * RG), 0,
                     s, xpart, nx, V * D, x0a);
  DCNR_LAUNCH_CHECK();
  FinalArgs fa;
  memset(&fa, 0, sizeof(fa));
  fa.cp = cp;
  for (int l = 0; l < L; ++l) { fa.dw[l] = gr.dw[l]; fa.db[l] = gr.db[l]; }
  fa.dwf = gr.dwf_cross; fa.dbf = gr.dbf;
  fa.D = D; fa.L = L; fa.accumulate = accumulate;
  hipLaunchKernelGGL(cross_final_kernel, dim3((unsigned)cdiv(D, CT)), dim3(CT), 0, s, fa, x0a,
                     scal);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
