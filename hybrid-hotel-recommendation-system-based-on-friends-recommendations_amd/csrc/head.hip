// Logit head and BCE loss (train.py:169-170, 206, 224), and the fused
// multi-tensor Adam/AdamW step (train.py:201-204, 226).
#include "dcnr_internal.h"

#include <cmath>
#include <type_traits>

namespace dcnr {
namespace {
constexpr int NT = 256;

// zdeep[b] = sum_n X[b][n] * w[n]   (deep half of final_linear), wave per row
template <typename T>
__global__ __launch_bounds__(NT) void row_dot_kernel(const T* X, int ld, int N, const float* w,
                                                     int64_t B, float* out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (NT / WAVE);
  for (int64_t b = (int64_t)blockIdx.x * (NT / WAVE) + (threadIdx.x >> 6); b < B; b += nw) {
    float s = 0.f;
    for (int n = lane; n < N; n += WAVE) s += St<T>::ld(X + b * ld + n) * w[n];
    s = wave_sum(s);
    if (lane == 0) out[b] = s;
  }
}

// bf16 rows, N % 8 == 0, N <= 64 * CPL: 8 lanes per row, each lane CPL
// 16-byte chunks (chunks j, j+8, ... of 8 columns: 128 B contiguous per 8
// lanes and load), its w slice held in registers; 3-step lane-group sum.
template <int CPL>
__global__ __launch_bounds__(NT) void row_dot8_kernel(const bf16* X, int ld, int N, const float* w,
                                                      int64_t B, float* out) {
  const int lane = threadIdx.x & 63, g = lane >> 3, j = lane & 7;
  const int nch = N / 8;
  float wr[CPL][8];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = j + 8 * i;
    const float4 lo = c < nch ? reinterpret_cast<const float4*>(w + 8 * c)[0] : float4{0.f, 0.f, 0.f, 0.f};
    const float4 hi = c < nch ? reinterpret_cast<const float4*>(w + 8 * c)[1] : float4{0.f, 0.f, 0.f, 0.f};
    wr[i][0] = lo.x; wr[i][1] = lo.y; wr[i][2] = lo.z; wr[i][3] = lo.w;
    wr[i][4] = hi.x; wr[i][5] = hi.y; wr[i][6] = hi.z; wr[i][7] = hi.w;
  }
  const int64_t nwv = (int64_t)gridDim.x * (NT / WAVE);
  for (int64_t r0 = ((int64_t)blockIdx.x * (NT / WAVE) + (threadIdx.x >> 6)) * 8; r0 < B; r0 += nwv * 8) {
    const int64_t b = r0 + g;
    float sum = 0.f;
    if (b < B) {
      u32x4 v[CPL];
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const int c = j + 8 * i;
        v[i] = c < nch ? *reinterpret_cast<const u32x4*>(X + b * ld + 8 * c) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int i = 0; i < CPL; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sum += __uint_as_float(v[i][e] << 16) * wr[i][2 * e];
          sum += __uint_as_float(v[i][e] & 0xffff0000u) * wr[i][2 * e + 1];
        }
    }
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    if (j == 0 && b < B) out[b] = sum;
  }
}

__global__ void logits_kernel(const float* zdeep, const float* zc, const float* bf, int64_t B,
                              float* z) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) z[i] = (zdeep[i] + zc[i]) + bf[0];
}

// eval head from the last GEMM's per-wave partial dots: z = sum_p part[p][b]
// (fixed order) + zc + bf
__global__ void head_parts_kernel(const float* part, int np, const float* zc, const float* bf,
                                  int64_t B, float* z) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  float d = 0.f;
  for (int p = 0; p < np; ++p) d += part[p * B + i];
  z[i] = (d + zc[i]) + bf[0];
}

// stage 1: per block partial sum of the BCE terms (+ dz); stage 2: fixed-order sum
__global__ __launch_bounds__(NT) void bce_kernel(const float* z, const float* y, int64_t B,
                                                 float* dz, float scale, double* part) {
  __shared__ double red[NT];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < B; i += (int64_t)gridDim.x * NT) {
    float zz = z[i], yy = y[i];
    // max(z,0) - z*y + log1p(exp(-|z|))   (torch's binary_cross_entropy_with_logits)
    float l = fmaxf(zz, 0.f) - zz * yy + log1pf(expf(-fabsf(zz)));
    acc += (double)l;
    if (dz) dz[i] = scale * (1.f / (1.f + expf(-zz)) - yy) / (float)B;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// fixed-order (deterministic) sum of the per-block partials
__global__ __launch_bounds__(NT) void bce_final_kernel(const double* part, int n, int64_t B,
                                                       float* loss) {
  __shared__ double red[NT];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += NT) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)(red[0] / (double)B);
}

constexpr int MAXT = 48;   // (the batch is a kernel argument: <= 4 KB)
struct AdamBatch {
  float* p[MAXT]; const float* g[MAXT]; float* m[MAXT]; float* v[MAXT];
  const uint8_t* map[MAXT];   // null, or a byte per row: 0 = gradient row not stored (exactly 0)
  int64_t n[MAXT]; int64_t blk0[MAXT + 1];
  int rw[MAXT];               // row width (elements) of a mapped tensor
  int nt;
};
static_assert(sizeof(AdamBatch) <= 4096, "kernel argument size");

// torch.optim AdamW / Adam (the foreach form torch uses on a GPU), fp32, in
// torch's order of operations and roundings:
//   AdamW: p *= 1 - lr*wd ; Adam: g += wd*p          (_foreach_mul_ / add)
//   m = lerp(m, g, 1-b1) = m + (1-b1)*(g - m)        (_foreach_lerp_: one fma)
//   v = v*b2 ; v += ((1-b2)*g)*g                      (_foreach_mul_, _foreach_addcmul_)
//   p += ((-lr/bc1)*m) / (sqrt(v)/sqrt(bc2) + eps)    (_foreach_addcdiv_)
__device__ __forceinline__ void adam_elem(float& pp, float gg, float& mm, float& vv, float lr, float b1,
                                          float b2, float eps, float wd, float step_size,
                                          float bc2_sqrt, int decoupled) {
  // every fused multiply-add spelled out, no other contraction: the 16-B
  // path and the element path (a tensor's unaligned tail, a mapped table's
  // last partial group) then round alike -- left to the compiler they
  // differed by an ulp of v (v*b2 is rounded before the add, as
  // torch's mul_ then addcmul_ do)
#pragma clang fp contract(off)
  if (decoupled) pp = pp * (1.f - lr * wd);
  else if (wd != 0.f) gg = fmaf(wd, pp, gg);
  mm = fmaf(1.f - b1, gg - mm, mm);
  vv = vv * b2;
  vv = vv + ((1.f - b2) * gg) * gg;
  const float denom = sqrtf(vv) / bc2_sqrt + eps;
  pp = pp + (-step_size * mm) / denom;
}

// One thread per 4 consecutive elements (16-B loads and stores where the
// tensor's four arrays are 16-B aligned, else element by element).
__global__ __launch_bounds__(NT) void adam_kernel(AdamBatch ab, float lr, float b1, float b2,
                                                  float eps, float wd, float step_size,
                                                  float bc2_sqrt, int decoupled) {
  int t = 0;
  while (t + 1 < ab.nt && (int64_t)blockIdx.x >= ab.blk0[t + 1]) ++t;
  const int64_t i0 = ((int64_t)blockIdx.x - ab.blk0[t]) * (NT * 4) + threadIdx.x * 4;
  float* p = ab.p[t];
  const float* g = ab.g[t];
  float* m = ab.m[t];
  float* v = ab.v[t];
  const int64_t n = ab.n[t];
  if (i0 >= n) return;
  const uint8_t* map = ab.map[t];
  const uint32_t rw = (uint32_t)ab.rw[t];
  // an unmarked row's gradient is exactly 0 and is not read (the same
  // arithmetic as a stored +0: m, v decay, weight decay, the update); the
  // row index in 32 bits below 2^32 elements, in 64 above (a uniform branch)
  const bool wide = n > (int64_t)0xFFFFFFFFll;
  bool gr[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    gr[e] = !map || (i0 + e < n && map[wide ? (i0 + e) / (int64_t)rw : (int64_t)((uint32_t)(i0 + e) / rw)]);
  const bool vec = i0 + 4 <= n && ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0);
  if (vec) {
    float4 pp = *reinterpret_cast<const float4*>(p + i0);
    float4 mm = *reinterpret_cast<const float4*>(m + i0);
    float4 vv = *reinterpret_cast<const float4*>(v + i0);
    float4 gg = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gr[0] || gr[1] || gr[2] || gr[3]) {
      gg = *reinterpret_cast<const float4*>(g + i0);
      if (!gr[0]) gg.x = 0.f;
      if (!gr[1]) gg.y = 0.f;
      if (!gr[2]) gg.z = 0.f;
      if (!gr[3]) gg.w = 0.f;
    }
    adam_elem(pp.x, gg.x, mm.x, vv.x, lr, b1, b2, eps, wd, step_size, bc2_sqrt, decoupled);
    adam_elem(pp.y, gg.y, mm.y, vv.y, lr, b1, b2, eps, wd, step_size, bc2_sqrt, decoupled);
    adam_elem(pp.z, gg.z, mm.z, vv.z, lr, b1, b2, eps, wd, step_size, bc2_sqrt, decoupled);
    adam_elem(pp.w, gg.w, mm.w, vv.w, lr, b1, b2, eps, wd, step_size, bc2_sqrt, decoupled);
    *reinterpret_cast<float4*>(p + i0) = pp;
    *reinterpret_cast<float4*>(m + i0) = mm;
    *reinterpret_cast<float4*>(v + i0) = vv;
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t i = i0 + e;
    if (i >= n) break;
    float pp = p[i], gg = gr[e] ? g[i] : 0.f, mm = m[i], vv = v[i];
    adam_elem(pp, gg, mm, vv, lr, b1, b2, eps, wd, step_size, bc2_sqrt, decoupled);
    p[i] = pp; m[i] = mm; v[i] = vv;
  }
}

}  // namespace

dcnr_status row_dot(int precision, const void* X, int ld, int N, const float* w, int64_t B,
                    float* out, hipStream_t s) {
  if (B <= 0) return DCNR_OK;
  int64_t blocks = std::min<int64_t>(cdiv(B, NT / WAVE), 4096);
  if (precision == DCNR_PREC_BF16 && N % 8 == 0 && ld % 8 == 0 && N <= 512 &&
      ((uintptr_t)X & 15) == 0 && ((uintptr_t)w & 15) == 0) {
    const int64_t b8 = std::min<int64_t>(cdiv(B, 8 * (NT / WAVE)), 1024);
    if (N <= 256)
      hipLaunchKernelGGL(row_dot8_kernel<4>, dim3((unsigned)b8), dim3(NT), 0, s, (const bf16*)X, ld, N, w, B, out);
    else
      hipLaunchKernelGGL(row_dot8_kernel<8>, dim3((unsigned)b8), dim3(NT), 0, s, (const bf16*)X, ld, N, w, B, out);
  } else if (precision == DCNR_PREC_BF16)
    hipLaunchKernelGGL(row_dot_kernel<bf16>, dim3((unsigned)blocks), dim3(NT), 0, s,
                       (const bf16*)X, ld, N, w, B, out);
  else
    hipLaunchKernelGGL(row_dot_kernel<float>, dim3((unsigned)blocks), dim3(NT), 0, s,
                       (const float*)X, ld, N, w, B, out);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status head_logits(const float* zdeep, const float* zc, const float* bf, int64_t B,
                        float* logits, hipStream_t s) {
  if (B <= 0) return DCNR_OK;
  hipLaunchKernelGGL(logits_kernel, dim3((unsigned)cdiv(B, NT)), dim3(NT), 0, s, zdeep, zc, bf, B,
                     logits);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status head_parts(const float* part, int np, const float* zc, const float* bf, int64_t B,
                       float* logits, hipStream_t s) {
  if (B <= 0) return DCNR_OK;
  hipLaunchKernelGGL(head_parts_kernel, dim3((unsigned)cdiv(B, NT)), dim3(NT), 0, s, part, np, zc, bf,
                     B, logits);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

constexpr int BCE_BLOCKS = 512;
size_t bce_ws_bytes() { return BCE_BLOCKS * sizeof(double); }

dcnr_status bce(const float* z, const float* y, int64_t B, float* loss, float* dz, float scale,
                double* part, hipStream_t s) {
  int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(BCE_BLOCKS, cdiv(B, NT)));
  hipLaunchKernelGGL(bce_kernel, dim3(blocks), dim3(NT), 0, s, z, y, B, dz, scale, part);
  DCNR_LAUNCH_CHECK();
  hipLaunchKernelGGL(bce_final_kernel, dim3(1), dim3(NT), 0, s, part, blocks, B, loss);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status adam(int n, float* const* p, const float* const* g, float* const* m, float* const* v,
                 const int64_t* numel, float lr, float b1, float b2, float eps, float wd,
                 int64_t step, int decoupled, hipStream_t s, const uint8_t* const* row_map,
                 const int32_t* row_width) {
  double bc1 = 1.0 - std::pow((double)b1, (double)step);
  double bc2 = 1.0 - std::pow((double)b2, (double)step);
  float step_size = (float)(lr / bc1);
  float bc2_sqrt = (float)std::sqrt(bc2);
  for (int off = 0; off < n; off += MAXT) {
    AdamBatch ab;
    ab.nt = std::min(MAXT, n - off);
    ab.blk0[0] = 0;
    for (int i = 0; i < ab.nt; ++i) {
      ab.p[i] = p[off + i]; ab.g[i] = g[off + i]; ab.m[i] = m[off + i]; ab.v[i] = v[off + i];
      ab.n[i] = numel[off + i];
      ab.map[i] = row_map ? row_map[off + i] : nullptr;
      ab.rw[i] = ab.map[i] ? row_width[off + i] : 1;
      ab.blk0[i + 1] = ab.blk0[i] + cdiv(ab.n[i], NT * 4);
    }
    int64_t blocks = ab.blk0[ab.nt];
    if (blocks == 0) continue;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(NT), 0, s, ab, lr, b1, b2, eps,
                       wd, step_size, bc2_sqrt, decoupled);
    DCNR_LAUNCH_CHECK();
  }
  return DCNR_OK;
}

}  // namespace dcnr
