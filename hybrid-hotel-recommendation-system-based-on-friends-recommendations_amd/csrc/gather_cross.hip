// Embedding gathers + x0 assembly + the cross stack, forward and backward, one
// 64-lane wave per sample row (gfx950).
//
// Forward  (DCN_RecSys.forward, train.py:156-159 and 167-168):
//   x0[b] = [U[u_b] | I[i_b] | C_0[c_b0] ... C_{K-1}[c_b,K-1] | num_b]   (bit-exact fp32 gather)
//   x_{l+1} = x_l + x_l * (x_l . w_l) + b_l                               (CrossLayer, train.py:96-99)
//   zc[b] = w_f[H:] . x_L       (the cross half of final_linear, train.py:169-170)
// The cross output itself is never written: the head only needs its dot with
// w_f.  x0 is written once, in the deep tower's storage type (A operand of the
// initial Linear).
//
// Backward re-gathers x0 in fp32 and recomputes the (cheap) cross forward in
// registers instead of saving per-layer activations:
//   g_L = dz * w_f[H:];  dx_l = g(1+s_l) + (g.x_l) w_l;  dw_l += (g.x_l) x_l;  db_l += g
//   dx0 = dx0_cross + dx0_deep  ->  dense embedding grads by row scatter-add
//   (embedding_dense_backward semantics; fp32 atomics, 128-B row segments).
// The x_l . w_l and g . x_l dots are wave reductions (xor shuffles).
#include "dcnr_internal.h"

namespace dcnr {
namespace {

constexpr int NT = 256;
constexpr int WPB = NT / WAVE;
constexpr int NUM_TAB = -1, NO_ELEM = -2;

struct TabLds {
  const float* tab[66];
  float* grad[66];
  int rows[66];
  int width[66];
};

template <int RM>
__device__ __forceinline__ void lane_map(const GatherDesc& g, int lane, int (&tab)[RM],
                                         int (&col)[RM]) {
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    int e = lane + WAVE * r;
    tab[r] = NO_ELEM;
    col[r] = 0;
    if (e < g.D) {
      int off = 0, t = 0;
      for (; t < g.n_tab; ++t) {
        if (e < off + g.width[t]) break;
        off += g.width[t];
      }
      tab[r] = t < g.n_tab ? t : NUM_TAB;
      col[r] = e - off;
    }
  }
}

// lanes < n_tab hold the (clamped) row index of table `lane` for sample b
__device__ __forceinline__ int load_ids(const GatherDesc& g, const int64_t* user,
                                        const int64_t* item, const int64_t* cat, int64_t b,
                                        int lane, int* err, int check) {
  int id = 0;
  if (lane < g.n_tab) {
    int64_t raw = lane == 0 ? user[b] : lane == 1 ? item[b]
                                                  : cat[b * (g.n_tab - 2) + (lane - 2)];
    int64_t n = g.rows[lane];
    if (raw < 0 || raw >= n) {
      if (check && err) atomicOr(err, 1);
      raw = raw < 0 ? 0 : n - 1;
    }
    id = (int)raw;
  }
  return id;
}

template <int RM>
__device__ __forceinline__ void gather_row(const GatherDesc& g, const TabLds& tl,
                                           const float* num, int64_t b, int myid,
                                           const int (&tab)[RM], const int (&col)[RM],
                                           int (&ids)[RM], float (&x)[RM]) {
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    int t = tab[r];
    int id = __shfl(myid, t >= 0 ? t : 0, WAVE);
    ids[r] = id;
    float v = 0.f;
    if (t >= 0) v = tl.tab[t][(int64_t)id * tl.width[t] + col[r]];
    else if (t == NUM_TAB) v = num[b * g.n_num + col[r]];
    x[r] = v;
  }
}

template <typename T, int RM>
__global__ __launch_bounds__(NT) void gather_cross_fwd_kernel(GatherDesc g, CrossParams cp,
                                                               const int64_t* user,
                                                               const int64_t* item,
                                                               const int64_t* cat,
                                                               const float* num, int64_t B, T* x0,
                                                               int ldx, float* zc, int* err,
                                                               int check) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  const int D = g.D, L = cp.L;
  float* sw = smem;              // [L][D]
  float* sb = sw + L * D;        // [L][D]
  float* swf = sb + L * D;       // [D]
  for (int i = threadIdx.x; i < L * D; i += NT) {
    sw[i] = cp.w[i / D][i % D];
    sb[i] = cp.b[i / D][i % D];
  }
  for (int i = threadIdx.x; i < D; i += NT) swf[i] = cp.wf_cross[i];
  for (int i = threadIdx.x; i < g.n_tab; i += NT) {
    tl.tab[i] = g.tab[i];
    tl.width[i] = g.width[i];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  int tab[RM], col[RM], ids[RM];
  lane_map<RM>(g, lane, tab, col);
  float x[RM];
  const int64_t nw = (int64_t)gridDim.x * WPB;
  for (int64_t b = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6); b < B; b += nw) {
    int myid = load_ids(g, user, item, cat, b, lane, err, check);
    gather_row<RM>(g, tl, num, b, myid, tab, col, ids, x);
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      int e = lane + WAVE * r;
      if (e < ldx) St<T>::st(x0 + b * ldx + e, x[r]);  // pad columns get 0
    }
    for (int l = 0; l < L; ++l) {
      float d = 0.f;
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        int e = lane + WAVE * r;
        if (e < D) d += x[r] * sw[l * D + e];
      }
      float s = wave_sum(d);
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        int e = lane + WAVE * r;
        if (e < D) x[r] = (x[r] + x[r] * s) + sb[l * D + e];
      }
    }
    float z = 0.f;
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      int e = lane + WAVE * r;
      if (e < D) z += x[r] * swf[e];
    }
    z = wave_sum(z);
    if (lane == 0) zc[b] = z;
  }
}

// part layout per wave: [L][D] dw | [L][D] db | [D] dwf | [1] dbf
template <int RM, int L>
__global__ __launch_bounds__(NT) void cross_bwd_kernel(GatherDesc g, CrossBwdParams p,
                                                        const int64_t* user, const int64_t* item,
                                                        const int64_t* cat, const float* num,
                                                        const float* dz, int64_t B,
                                                        const float* dx0_deep, int ld_dx,
                                                        float* part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  const int D = g.D;
  float* sw = smem;
  float* sb = sw + L * D;
  float* swf = sb + L * D;
  for (int i = threadIdx.x; i < L * D; i += NT) {
    sw[i] = p.cp.w[i / D][i % D];
    sb[i] = p.cp.b[i / D][i % D];
  }
  for (int i = threadIdx.x; i < D; i += NT) swf[i] = p.cp.wf_cross[i];
  for (int i = threadIdx.x; i < g.n_tab; i += NT) {
    tl.tab[i] = g.tab[i];
    tl.grad[i] = p.emb_grad[i];
    tl.width[i] = g.width[i];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  int tab[RM], col[RM], ids[RM];
  lane_map<RM>(g, lane, tab, col);
  float xs[L + 1][RM];
  float s[L > 0 ? L : 1];
  float dwa[L > 0 ? L : 1][RM], dba[L > 0 ? L : 1][RM], dwfa[RM];
  float dbf = 0.f;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    dwfa[r] = 0.f;
#pragma unroll
    for (int l = 0; l < L; ++l) { dwa[l][r] = 0.f; dba[l][r] = 0.f; }
  }
  const int64_t wid = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * WPB;
  for (int64_t b = wid; b < B; b += nw) {
    int myid = load_ids(g, user, item, cat, b, lane, nullptr, 0);
    gather_row<RM>(g, tl, num, b, myid, tab, col, ids, xs[0]);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      float d = 0.f;
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        int e = lane + WAVE * r;
        if (e < D) d += xs[l][r] * sw[l * D + e];
      }
      s[l] = wave_sum(d);
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        int e = lane + WAVE * r;
        xs[l + 1][r] = e < D ? (xs[l][r] + xs[l][r] * s[l]) + sb[l * D + e] : 0.f;
      }
    }
    const float dd = dz[b];
    dbf += dd;
    float gr[RM];
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      int e = lane + WAVE * r;
      gr[r] = e < D ? dd * swf[e] : 0.f;
      dwfa[r] += dd * xs[L][r];
    }
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
      float d = 0.f;
#pragma unroll
      for (int r = 0; r < RM; ++r) d += gr[r] * xs[l][r];
      float gx = wave_sum(d);
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        int e = lane + WAVE * r;
        dba[l][r] += gr[r];
        dwa[l][r] += gx * xs[l][r];
        gr[r] = e < D ? gr[r] * (1.f + s[l]) + gx * sw[l * D + e] : 0.f;
      }
    }
    // dx0 = cross part + deep part; scatter into the dense embedding grads
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      int t = tab[r];
      if (t >= 0) {
        int e = lane + WAVE * r;
        float v = gr[r] + dx0_deep[b * ld_dx + e];
        atomicAdd(tl.grad[t] + (int64_t)ids[r] * tl.width[t] + col[r], v);
      }
    }
  }
  // block-level partial: the 4 waves add into LDS in fixed wave order
  // (deterministic), then one coalesced store per block
  const int stride = (2 * L + 1) * D + 1;
  float* red = swf + D;   // [stride] after the weight region
  const int w = threadIdx.x >> 6;
  for (int ww = 0; ww < WPB; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        int e = lane + WAVE * r;
        if (e >= D) continue;
#pragma unroll
        for (int l = 0; l < L; ++l) {
          red[l * D + e] = (ww ? red[l * D + e] : 0.f) + dwa[l][r];
          red[(L + l) * D + e] = (ww ? red[(L + l) * D + e] : 0.f) + dba[l][r];
        }
        red[2 * L * D + e] = (ww ? red[2 * L * D + e] : 0.f) + dwfa[r];
      }
      if (lane == 0) red[(2 * L + 1) * D] = (ww ? red[(2 * L + 1) * D] : 0.f) + dbf;
    }
    __syncthreads();
  }
  float* mp = part + (int64_t)blockIdx.x * stride;
  for (int i = threadIdx.x; i < stride; i += NT) mp[i] = red[i];
}

// reduce per-block partials -> grads (8 elements x 32 lanes per block, fixed order)
__global__ __launch_bounds__(NT) void cross_reduce_kernel(const float* part, int64_t nb, int D,
                                                          int L, CrossBwdParams p, int accumulate) {
  __shared__ float red[32][8];
  const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int64_t stride = (int64_t)(2 * L + 1) * D + 1;
  const int64_t i = (int64_t)blockIdx.x * 8 + tx;
  float s = 0.f;
  if (i < stride)
    for (int64_t w = ty; w < nb; w += 32) s += part[w * stride + i];
  red[ty][tx] = s;
  __syncthreads();
  for (int o = 16; o > 0; o >>= 1) {
    if (ty < o) red[ty][tx] += red[ty + o][tx];
    __syncthreads();
  }
  if (ty != 0 || i >= stride) return;
  s = red[0][tx];
  float* dst;
  if (i < (int64_t)L * D) dst = p.dw[i / D] + i % D;
  else if (i < (int64_t)2 * L * D) dst = p.db[(i - L * D) / D] + (i - L * D) % D;
  else if (i < stride - 1) dst = p.dwf_cross + (i - 2 * L * D);
  else dst = p.dbf;
  *dst = accumulate ? *dst + s : s;
}

template <typename T, int RM>
dcnr_status launch_fwd(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                       const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                       void* x0, int ldx, float* zc, int* err, int check, hipStream_t s) {
  size_t lds = (size_t)(2 * cp.L + 1) * g.D * sizeof(float);
  int64_t blocks = std::min<int64_t>(cdiv(B, WPB), 256 * 8);
  hipLaunchKernelGGL((gather_cross_fwd_kernel<T, RM>), dim3((unsigned)blocks), dim3(NT), lds, s, g,
                     cp, user, item, cat, num, B, (T*)x0, ldx, zc, err, check);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

template <int RM, int L>
dcnr_status launch_bwd(const GatherDesc& g, const CrossBwdParams& p, const int64_t* user,
                       const int64_t* item, const int64_t* cat, const float* num, const float* dz,
                       int64_t B, const float* dx0, int ld_dx, float* part, int64_t nw,
                       hipStream_t s) {
  size_t lds = (size_t)(2 * (2 * L + 1) * g.D + 1) * sizeof(float);
  hipLaunchKernelGGL((cross_bwd_kernel<RM, L>), dim3((unsigned)nw), dim3(NT), lds, s, g, p,
                     user, item, cat, num, dz, B, dx0, ld_dx, part);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

template <int RM>
dcnr_status dispatch_bwd_L(int L, const GatherDesc& g, const CrossBwdParams& p,
                           const int64_t* user, const int64_t* item, const int64_t* cat,
                           const float* num, const float* dz, int64_t B, const float* dx0,
                           int ld_dx, float* part, int64_t nw, hipStream_t s) {
  switch (L) {
#define CASE(n) \
  case n: return launch_bwd<RM, n>(g, p, user, item, cat, num, dz, B, dx0, ld_dx, part, nw, s);
    CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7)
#undef CASE
  }
  set_error("cross: n_cross_layers=%d unsupported (max 7)", L);
  return DCNR_UNSUPPORTED_SHAPE;
}

constexpr int64_t BWD_BLOCKS = 2048;  // x4 waves: 32 waves/CU of latency hiding

}  // namespace

size_t cross_bwd_part_elems(int D, int L) { return (size_t)BWD_BLOCKS * ((2 * L + 1) * D + 1); }

dcnr_status gather_cross_fwd(int precision, const GatherDesc& g, const CrossParams& cp,
                             const int64_t* user, const int64_t* item, const int64_t* cat,
                             const float* num, int64_t B, void* x0, int ldx, float* zc, int* err,
                             int check, hipStream_t s) {
  if (B <= 0) return DCNR_OK;
  if (g.D > 16 * WAVE || cp.L > 8 || g.n_tab > 66) {
    set_error("gather: unsupported D=%d / n_cross=%d / tables=%d", g.D, cp.L, g.n_tab);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  bool small = g.D <= 8 * WAVE && ldx <= 8 * WAVE;
  if (precision == DCNR_PREC_BF16)
    return small ? launch_fwd<bf16, 8>(g, cp, user, item, cat, num, B, x0, ldx, zc, err, check, s)
                 : launch_fwd<bf16, 16>(g, cp, user, item, cat, num, B, x0, ldx, zc, err, check, s);
  return small ? launch_fwd<float, 8>(g, cp, user, item, cat, num, B, x0, ldx, zc, err, check, s)
               : launch_fwd<float, 16>(g, cp, user, item, cat, num, B, x0, ldx, zc, err, check, s);
}

dcnr_status cross_bwd_scatter(const GatherDesc& g, const CrossBwdParams& p, const int64_t* user,
                              const int64_t* item, const int64_t* cat, const float* num,
                              const float* dz, int64_t B, const float* dx0_deep, int ld_dx,
                              float* part, size_t part_elems, int accumulate, hipStream_t s) {
  const int L = p.cp.L, D = g.D;
  if (part_elems < cross_bwd_part_elems(D, L)) {
    set_error("cross_bwd: partial buffer too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  if (D > 16 * WAVE) {
    set_error("cross_bwd: D=%d unsupported", D);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  dcnr_status st = D <= 8 * WAVE
                       ? dispatch_bwd_L<8>(L, g, p, user, item, cat, num, dz, B, dx0_deep, ld_dx,
                                           part, BWD_BLOCKS, s)
                       : dispatch_bwd_L<16>(L, g, p, user, item, cat, num, dz, B, dx0_deep, ld_dx,
                                            part, BWD_BLOCKS, s);
  if (st != DCNR_OK) return st;
  int64_t stride = (int64_t)(2 * L + 1) * D + 1;
  hipLaunchKernelGGL(cross_reduce_kernel, dim3((unsigned)cdiv(stride, 8)), dim3(NT), 0, s, part,
                     BWD_BLOCKS, D, L, p, accumulate);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
