// Embedding gathers + x0 assembly + the cross stack, forward and backward, and
// the dense embedding gradient (gfx950, 64-lane waves, one wave per sample row).
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
//   dx0 = dx0_cross + dx0_deep  ->  dense embedding grads (embedding_dense_backward)
//
// Latency structure (the gathers are dependent loads: id -> row): a block
// stages the ids of a tile of samples in LDS with coalesced loads, then each
// wave issues the row loads of several samples back to back (unconditional
// loads at clamped addresses, so no per-element branch serialises them)
// before computing any of them.
//
// Embedding gradients: every table row segment is added with no-return fp32
// atomics (128-B row segments, executed memory-side and overlapped with the
// kernel's own work).  Measured alternative (kept out): privatising the small
// categorical tables in LDS (per-sample dcat stores + an LDS-atomic per-table
// pass) cost 285 us against +30 us for the inline atomics at cfg3 (an early
// version of this kernel; on the current one the scatter costs 142 of 306 us,
// tools/gather_lab.hip modes 0 / 8, so the privatised form is worth a retry).
#include "dcnr_internal.h"

#include <cstring>

// tools/gather_lab.hip rebuilds this file with GC_LAB_MODE bits set to time
// parts of the kernels in isolation (forward 1: no x0 stores, 2: no cross
// compute, 4: no row loads; backward 8: no gradient scatter, 16: no cross
// compute).  The library always builds mode 0.
#ifndef GC_LAB_MODE
#define GC_LAB_MODE 0
#endif

namespace dcnr {
namespace {

constexpr int NT = 256;
constexpr int WPB = NT / WAVE;
constexpr int NUM_TAB = -1, NO_ELEM = -2;

struct TabLds {
  const float* tab[MAX_TABLES];
  float* grad[MAX_TABLES];
  int rows[MAX_TABLES];
  int width[MAX_TABLES];
  int off[MAX_TABLES];
};

// Per-lane element map of a sample row: element e = lane + 64 r.
template <int RM>
struct LaneMap {
  const float* base[RM];  // row-0 address of this element's source (or a valid dummy)
  int stride[RM];         // source row stride (floats)
  int tab[RM];            // table index, NUM_TAB or NO_ELEM
  int col[RM];            // column inside the table row
};

template <int RM>
__device__ __forceinline__ void make_lanes(const GatherDesc& g, const TabLds& tl, const float* num,
                                           int lane, LaneMap<RM>& m) {
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int e = lane + WAVE * r;
    int t = NO_ELEM, col = 0;
    if (e < g.D) {
      t = NUM_TAB;
      col = e - (g.D - g.n_num);
      for (int q = 0; q < g.n_tab; ++q)
        if (e >= tl.off[q] && e < tl.off[q] + tl.width[q]) { t = q; col = e - tl.off[q]; }
    }
    m.tab[r] = t;
    m.col[r] = col;
    m.base[r] = t >= 0 ? tl.tab[t] + col : (t == NUM_TAB ? num + col : tl.tab[0]);
    m.stride[r] = t >= 0 ? tl.width[t] : (t == NUM_TAB ? g.n_num : 0);
  }
}

// Stage the clamped row ids of samples [b0, b0 + S) into LDS ids[S][n_tab]
// (tail samples get id 0, a valid row).  Coalesced: consecutive threads read
// consecutive index entries.
__device__ __forceinline__ void stage_ids(const GatherDesc& g, const TabLds& tl,
                                          const int64_t* user, const int64_t* item,
                                          const int64_t* cat, int64_t b0, int S, int64_t B,
                                          int* ids, int* err, int check) {
  const int nt = g.n_tab;
  for (int e = threadIdx.x; e < S * nt; e += NT) {
    const int s = e / nt, t = e - s * nt;
    const int64_t b = b0 + s;
    int id = 0;
    if (b < B) {
      int64_t raw = t == 0 ? user[b] : t == 1 ? item[b] : cat[b * (nt - 2) + (t - 2)];
      const int64_t n = tl.rows[t];
      if (raw < 0 || raw >= n) {
        if (check && err) atomicOr(err, 1);
        raw = raw < 0 ? 0 : n - 1;
      }
      id = (int)raw;
    }
    ids[e] = id;
  }
}

// x0 row of tile-sample s (global row b, clamped for the tail): RM loads, all
// unconditional
template <int RM>
__device__ __forceinline__ void load_row(const LaneMap<RM>& m, const int* ids_s, int64_t bc,
                                         float (&x)[RM]) {
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int t = m.tab[r];
    const int64_t row = t >= 0 ? (int64_t)ids_s[t] : (t == NUM_TAB ? bc : 0);
    x[r] = m.base[r][row * m.stride[r]];
  }
#pragma unroll
  for (int r = 0; r < RM; ++r) x[r] = m.tab[r] == NO_ELEM ? 0.f : x[r];
}

__device__ __forceinline__ void fill_tab_lds(const GatherDesc& g, TabLds& tl, float* const* grad) {
  for (int i = threadIdx.x; i < g.n_tab; i += NT) {
    tl.tab[i] = g.tab[i];
    tl.rows[i] = (int)g.rows[i];
    tl.width[i] = g.width[i];
    tl.off[i] = g.off[i];
    tl.grad[i] = grad ? grad[i] : nullptr;
  }
}

// ---------------------------------------------------------------- forward
// SPW samples per wave per tile, all row loads of a tile issued before use.
template <typename T, int RM, int SPW>
__global__ __launch_bounds__(NT) void gather_cross_fwd_kernel(GatherDesc g, CrossParams cp,
                                                               const int64_t* user,
                                                               const int64_t* item,
                                                               const int64_t* cat,
                                                               const float* num, int64_t B, T* x0,
                                                               int ldx, float* zc, int* err,
                                                               int check, float* cross, int ldc) {
  constexpr int S = SPW * WPB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  const int D = g.D, L = cp.L;
  float* sw = smem;              // [L][D]
  float* sb = sw + L * D;        // [L][D]
  float* swf = sb + L * D;       // [D]
  int* ids = reinterpret_cast<int*>(swf + D);  // [S][n_tab]
  // per-wave bf16 staging row for the x0 store (16-B aligned)
  bf16* stage = reinterpret_cast<bf16*>(smem + ((L * D * 2 + D + S * g.n_tab + 3) & ~3)) +
                (threadIdx.x >> 6) * RM * WAVE;
  static_assert(SPW == 4, "the forward reduces 4 samples per wave together");
  for (int i = threadIdx.x; i < L * D; i += NT) {
    sw[i] = cp.w[i / D][i % D];
    sb[i] = cp.b[i / D][i % D];
  }
  for (int i = threadIdx.x; i < D; i += NT) swf[i] = cp.wf_cross[i];
  fill_tab_lds(g, tl, nullptr);
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  LaneMap<RM> m;
  make_lanes<RM>(g, tl, num, lane, m);
  const int64_t ntiles = (B + S - 1) / S;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * S;
    __syncthreads();  // the previous tile's ids are consumed
    stage_ids(g, tl, user, item, cat, b0, S, B, ids, err, check);
    __syncthreads();
    float x[SPW][RM];
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int s = w * SPW + u;
      const int64_t b = b0 + s;
      if constexpr (!(GC_LAB_MODE & 4))
        load_row<RM>(m, ids + s * g.n_tab, b < B ? b : B - 1, x[u]);
      else
        for (int r = 0; r < RM; ++r) x[u][r] = (float)ids[s * g.n_tab + (r & 1)];
    }
    // x0 in the deep tower's storage type.  bf16: staged through this wave's
    // LDS row so every lane stores 16 contiguous bytes (8 columns)
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int64_t b = b0 + w * SPW + u;
      if (x0 == nullptr) continue;
      if constexpr (!(GC_LAB_MODE & 1)) {
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            const int e = lane + WAVE * r;
            if (e < ldx) stage[e] = (bf16)x[u][r];   // pad columns get 0
          }
          if (b < B && lane * 8 < ldx)
            *reinterpret_cast<uint4*>(x0 + b * ldx + lane * 8) =
                *reinterpret_cast<const uint4*>(stage + lane * 8);
          if constexpr (RM > 8)
            if (b < B && (lane + 64) * 8 < ldx)
              *reinterpret_cast<uint4*>(x0 + b * ldx + (lane + 64) * 8) =
                  *reinterpret_cast<const uint4*>(stage + (lane + 64) * 8);
        } else {
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            const int e = lane + WAVE * r;
            if (b < B && e < ldx) St<T>::st(x0 + b * ldx + e, x[u][r]);
          }
        }
      }
    }
    // cross stack: the SPW (=4) samples' dot products are reduced together
    if constexpr (!(GC_LAB_MODE & 2)) {
      for (int l = 0; l < L; ++l) {
        float d[SPW];
#pragma unroll
        for (int u = 0; u < SPW; ++u) {
          d[u] = 0.f;
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            const int e = lane + WAVE * r;
            if (e < D) d[u] += x[u][r] * sw[l * D + e];
          }
        }
        float sl[SPW];
        wave_sum4(d[0], d[1], d[2], d[3], sl[0], sl[1], sl[2], sl[3]);
#pragma unroll
        for (int u = 0; u < SPW; ++u)
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            const int e = lane + WAVE * r;
            if (e < D) x[u][r] = (x[u][r] + x[u][r] * sl[u]) + sb[l * D + e];
          }
      }
    }
    if (cross) {
#pragma unroll
      for (int u = 0; u < SPW; ++u) {
        const int64_t b = b0 + w * SPW + u;
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          const int e = lane + WAVE * r;
          if (b < B && e < ldc) cross[b * ldc + e] = x[u][r];
        }
      }
    }
    if (!zc) continue;
    float z[SPW];
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      z[u] = 0.f;
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        const int e = lane + WAVE * r;
        if (e < D) z[u] += x[u][r] * swf[e];
      }
    }
    float zs[SPW];
    wave_sum4(z[0], z[1], z[2], z[3], zs[0], zs[1], zs[2], zs[3]);
    if (lane < SPW) {
      const int64_t b = b0 + w * SPW + lane;
      const float zv = lane == 0 ? zs[0] : lane == 1 ? zs[1] : lane == 2 ? zs[2] : zs[3];
      if (b < B) zc[b] = zv;
    }
  }
}

// ------------------------------------------------ forward, 16-byte lanes
// Fast path when every table width, n_num and D are multiples of 4 (cfg2/cfg3:
// 32-wide tables, 8 dense features, D = 456): lane l of a wave owns the float4
// chunk c = l + 64 r (elements 4c..4c+3) of a sample row, r < R4, so a 32-wide
// table row is 8 lanes x 16 B and the whole x0 row of 456 floats is R4 = 2
// dwordx4 gathers.  Each wave owns SPW consecutive samples per tile.  It loads
// their row ids itself, one int64 per lane, coalesced (lane j: sample j / n_tab,
// table j % n_tab).  ds_bpermute hands each lane the id of its table.  No block
// barrier is taken inside the loop, and the next tile's ids are loaded before
// this tile's rows are consumed (one-tile software pipeline).
typedef __attribute__((ext_vector_type(4))) float v4f;

__device__ __forceinline__ float dot4(v4f a, v4f b) {
  return ((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3];
}

template <int IDR>
__device__ __forceinline__ int lane_id_of(const int (&idr)[IDR], int src) {
  const int v0 = __builtin_amdgcn_ds_bpermute((src & 63) << 2, idr[0]);
  if constexpr (IDR == 1) return v0;
  else {
    const int v1 = __builtin_amdgcn_ds_bpermute((src & 63) << 2, idr[1]);
    return src < 64 ? v0 : v1;
  }
}

template <int R4, int SPW, int IDR, int X0BF16>
__global__ __launch_bounds__(NT) void gather_cross_v4_kernel(GatherDesc g, CrossParams cp,
                                                             const int64_t* user,
                                                             const int64_t* item,
                                                             const int64_t* cat, const float* num,
                                                             int64_t B, GcOut out, int* err,
                                                             int check) {
  static_assert(SPW % 4 == 0, "dot products are reduced 4 samples at a time");
  constexpr int C = R4 * WAVE;       // float4 chunks per image
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  const int D = g.D, L = cp.L, nt = g.n_tab;
  v4f* sw = reinterpret_cast<v4f*>(smem);   // [L][C]  w_l chunks (0 past D)
  v4f* sb = sw + L * C;                     // [L][C]  b_l
  v4f* swf = sb + L * C;                    // [C]     w_f[H:]
  for (int i = threadIdx.x; i < (2 * L + 1) * C * 4; i += NT) {
    const int l = i / (C * 4), e = i % (C * 4);
    float v = 0.f;
    if (e < D) v = l < L ? cp.w[l][e] : l < 2 * L ? cp.b[l - L][e] : cp.wf_cross[e];
    smem[i] = v;
  }
  fill_tab_lds(g, tl, nullptr);
  __syncthreads();

  const int lane = threadIdx.x & 63;
  // chunk map of this lane
  const float* base[R4];
  int stride[R4], tab[R4];
#pragma unroll
  for (int r = 0; r < R4; ++r) {
    const int e = 4 * (lane + WAVE * r);
    int t = NO_ELEM, col = 0;
    if (e < D) {
      t = NUM_TAB;
      col = e - (D - g.n_num);
      for (int q = 0; q < nt; ++q)
        if (e >= tl.off[q] && e < tl.off[q] + tl.width[q]) { t = q; col = e - tl.off[q]; }
    }
    tab[r] = t;
    base[r] = t >= 0 ? tl.tab[t] + col : (t == NUM_TAB ? num + col : tl.tab[0]);
    stride[r] = t >= 0 ? tl.width[t] : (t == NUM_TAB ? g.n_num : 0);
  }
  // id map of this lane: id slot j = lane + 64 q -> (sample j / nt, table j % nt)
  int ju[IDR], jt[IDR];
  int64_t jrows[IDR];
#pragma unroll
  for (int q = 0; q < IDR; ++q) {
    const int j = lane + WAVE * q;
    ju[q] = j / nt;
    jt[q] = j % nt;
    jrows[q] = tl.rows[jt[q]];
  }
  auto load_ids = [&](int64_t b0, int (&idr)[IDR]) {
#pragma unroll
    for (int q = 0; q < IDR; ++q) {
      const int64_t b = b0 + ju[q];
      const bool ok = ju[q] < SPW && b < B;
      const int t = jt[q];
      const int64_t bc = ok ? b : 0;
      const int64_t* src = t == 0 ? user + bc : t == 1 ? item + bc : cat + bc * (nt - 2) + (t - 2);
      int64_t raw = ok ? *src : 0;
      if (raw < 0 || raw >= jrows[q]) {
        if (check && err) atomicOr(err, 1);
        raw = raw < 0 ? 0 : jrows[q] - 1;
      }
      idr[q] = (int)raw;
    }
  };

  const int64_t ntiles = (B + SPW - 1) / SPW;
  const int64_t wave_id = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int64_t n_waves = (int64_t)gridDim.x * WPB;
  int idc[IDR];
  if (wave_id < ntiles) load_ids(wave_id * SPW, idc);
  for (int64_t tile = wave_id; tile < ntiles; tile += n_waves) {
    const int64_t b0 = tile * SPW;
    v4f x[SPW][R4];
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int64_t bc = b0 + u < B ? b0 + u : B - 1;
#pragma unroll
      for (int r = 0; r < R4; ++r) {
        const int t = tab[r];
        const int id = lane_id_of<IDR>(idc, u * nt + (t >= 0 ? t : 0));
        const int64_t row = t >= 0 ? (int64_t)id : (t == NUM_TAB ? bc : 0);
        x[u][r] = *reinterpret_cast<const v4f*>(base[r] + row * stride[r]);
      }
    }
    if (tile + n_waves < ntiles) load_ids((tile + n_waves) * SPW, idc);
#pragma unroll
    for (int u = 0; u < SPW; ++u)
#pragma unroll
      for (int r = 0; r < R4; ++r)
        if (tab[r] == NO_ELEM) x[u][r] = v4f{0.f, 0.f, 0.f, 0.f};
    // x0 (A operand of the initial Linear), pad columns 0
    if (out.x0) {
#pragma unroll
      for (int u = 0; u < SPW; ++u) {
        const int64_t b = b0 + u;
#pragma unroll
        for (int r = 0; r < R4; ++r) {
          const int e = 4 * (lane + WAVE * r);
          if (b < B && e < out.ld_x0) {
            if constexpr (X0BF16) {
              bf16x4 h = {(bf16)x[u][r][0], (bf16)x[u][r][1], (bf16)x[u][r][2], (bf16)x[u][r][3]};
              *reinterpret_cast<bf16x4*>(static_cast<bf16*>(out.x0) + b * out.ld_x0 + e) = h;
            } else {
              *reinterpret_cast<v4f*>(static_cast<float*>(out.x0) + b * out.ld_x0 + e) = x[u][r];
            }
          }
        }
      }
    }
    // cross stack (CrossLayer, train.py:96-99): x <- (x + x*(x.w)) + b
    for (int l = 0; l < L; ++l) {
      v4f wv[R4], bv[R4];
#pragma unroll
      for (int r = 0; r < R4; ++r) {
        wv[r] = sw[l * C + lane + WAVE * r];
        bv[r] = sb[l * C + lane + WAVE * r];
      }
#pragma unroll
      for (int u0 = 0; u0 < SPW; u0 += 4) {
        float d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = 0.f;
#pragma unroll
          for (int r = 0; r < R4; ++r) d[k] += dot4(x[u0 + k][r], wv[r]);
        }
        float s[4];
        wave_sum4(d[0], d[1], d[2], d[3], s[0], s[1], s[2], s[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int r = 0; r < R4; ++r) x[u0 + k][r] = (x[u0 + k][r] + x[u0 + k][r] * s[k]) + bv[r];
      }
    }
    if (out.cross) {
#pragma unroll
      for (int u = 0; u < SPW; ++u) {
        const int64_t b = b0 + u;
#pragma unroll
        for (int r = 0; r < R4; ++r) {
          const int e = 4 * (lane + WAVE * r);
          if (b < B && e < out.ld_cross)
            __builtin_nontemporal_store(x[u][r], reinterpret_cast<v4f*>(out.cross + b * out.ld_cross + e));
        }
      }
    }
    if (out.zc) {
      v4f fv[R4];
#pragma unroll
      for (int r = 0; r < R4; ++r) fv[r] = swf[lane + WAVE * r];
#pragma unroll
      for (int u0 = 0; u0 < SPW; u0 += 4) {
        float z[4], zs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          z[k] = 0.f;
#pragma unroll
          for (int r = 0; r < R4; ++r) z[k] += dot4(x[u0 + k][r], fv[r]);
        }
        wave_sum4(z[0], z[1], z[2], z[3], zs[0], zs[1], zs[2], zs[3]);
        if (lane < 4) {
          const int64_t b = b0 + u0 + lane;
          const float zv = lane == 0 ? zs[0] : lane == 1 ? zs[1] : lane == 2 ? zs[2] : zs[3];
          if (b < B) out.zc[b] = zv;
        }
      }
    }
  }
}

// --------------------------------------------------------------- backward
// part layout per block: [L][D] dw | [L][D] db | [D] dwf | [1] dbf
// Per-lane transposed LDS images: element e = lane + 64r of a D-vector sits
// at [lane][r] (RM consecutive floats per lane: two ds_read_b128 per vector),
// zero for e >= D, so the math below needs no per-element bounds tests.
typedef float f2v __attribute__((ext_vector_type(2)));

template <int RM>
__device__ __forceinline__ void lds_vec(const float* img, int lane, f2v (&v)[RM / 2]) {
  const float4* p4 = reinterpret_cast<const float4*>(img + lane * RM);
#pragma unroll
  for (int i = 0; i < RM / 4; ++i) {
    const float4 t = p4[i];
    v[2 * i] = f2v{t.x, t.y};
    v[2 * i + 1] = f2v{t.z, t.w};
  }
}
template <int RM>
__device__ __forceinline__ void lds_store_vec(float* img, int lane, const f2v (&v)[RM / 2]) {
  float4* p4 = reinterpret_cast<float4*>(img + lane * RM);
#pragma unroll
  for (int i = 0; i < RM / 4; ++i)
    p4[i] = float4{v[2 * i][0], v[2 * i][1], v[2 * i + 1][0], v[2 * i + 1][1]};
}

template <int RM, int L, int SPW>
__global__ __launch_bounds__(NT, 2) void cross_bwd_kernel(GatherDesc g, CrossBwdParams p,
                                                        const int64_t* user, const int64_t* item,
                                                        const int64_t* cat, const float* num,
                                                        const float* dz, int64_t B,
                                                        const float* dx0_deep, int ld_dx,
                                                        float* part) {
  constexpr int S = SPW * WPB, V = RM * WAVE, H2 = RM / 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  const int D = g.D;
  float* sw = smem;                 // [L][V] transposed images
  float* sb = sw + L * V;           // [L][V]
  float* swf = sb + L * V;          // [V]
  float* red = swf + V;             // [(2L+1)D+1] block partial (16-B padded)
  int* ids = reinterpret_cast<int*>(red + (((2 * L + 1) * D + 1 + 3) & ~3));  // [S][n_tab]
  // per-wave cross activations x_0..x_{L-1} of the sample in flight (LDS
  // instead of registers: keeps the kernel at 2 waves/SIMD without spills)
  float* xsl = reinterpret_cast<float*>(ids + ((S * g.n_tab + 3) & ~3)) + (threadIdx.x >> 6) * L * V;
  for (int i = threadIdx.x; i < (2 * L + 1) * V; i += NT) {
    const int l = i / V, pos = i % V, ln = pos / RM, r = pos % RM, e = ln + WAVE * r;
    float v = 0.f;
    if (e < D) v = l < L ? p.cp.w[l][e] : l < 2 * L ? p.cp.b[l - L][e] : p.cp.wf_cross[e];
    sw[i] = v;
  }
  fill_tab_lds(g, tl, p.emb_grad);
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  LaneMap<RM> m;
  make_lanes<RM>(g, tl, num, lane, m);
  f2v dwa[L > 0 ? L : 1][H2], dba[L > 0 ? L : 1][H2], dwfa[H2];
  float dbf = 0.f;
#pragma unroll
  for (int h = 0; h < H2; ++h) {
    dwfa[h] = f2v{0.f, 0.f};
#pragma unroll
    for (int l = 0; l < L; ++l) { dwa[l][h] = f2v{0.f, 0.f}; dba[l][h] = f2v{0.f, 0.f}; }
  }
  const int64_t ntiles = (B + S - 1) / S;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * S;
    __syncthreads();
    stage_ids(g, tl, user, item, cat, b0, S, B, ids, nullptr, 0);
    __syncthreads();
    float x[SPW][RM], dd[SPW][RM], dzv[SPW];
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int s = w * SPW + u;
      const int64_t b = b0 + s;
      const int64_t bc = b < B ? b : B - 1;
      load_row<RM>(m, ids + s * g.n_tab, bc, x[u]);
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        const int e = lane + WAVE * r;
        dd[u][r] = dx0_deep[bc * ld_dx + (e < ld_dx ? e : 0)];
      }
      dzv[u] = dz[bc];
    }
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int s = w * SPW + u;
      const int64_t b = b0 + s;
      if (b >= B) break;
      float sl[L > 0 ? L : 1];
      f2v xc[H2];
#pragma unroll
      for (int h = 0; h < H2; ++h)   // elements past D are 0 (the images are 0 there too)
        xc[h] = f2v{m.tab[2 * h] != NO_ELEM ? x[u][2 * h] : 0.f,
                    m.tab[2 * h + 1] != NO_ELEM ? x[u][2 * h + 1] : 0.f};
#pragma unroll
      for (int l = 0; l < ((GC_LAB_MODE & 16) ? 0 : L); ++l) {
        lds_store_vec<RM>(xsl + l * V, lane, xc);
        f2v wv[H2], bv[H2];
        lds_vec<RM>(sw + l * V, lane, wv);
        lds_vec<RM>(sb + l * V, lane, bv);
        f2v d2 = f2v{0.f, 0.f};
#pragma unroll
        for (int h = 0; h < H2; ++h) d2 += xc[h] * wv[h];
        sl[l] = wave_sum_dpp(d2[0] + d2[1]);
        const f2v sv = f2v{sl[l], sl[l]};
#pragma unroll
        for (int h = 0; h < H2; ++h) xc[h] = (xc[h] + xc[h] * sv) + bv[h];
      }
      const float dzb = dzv[u];
      dbf += dzb;
      const f2v dzv2 = f2v{dzb, dzb};
      f2v gr[H2];
      {
        f2v fv[H2];
        lds_vec<RM>(swf, lane, fv);
#pragma unroll
        for (int h = 0; h < H2; ++h) {
          gr[h] = dzv2 * fv[h];
          dwfa[h] += dzv2 * xc[h];
        }
      }
#pragma unroll
      for (int l = ((GC_LAB_MODE & 16) ? -1 : L - 1); l >= 0; --l) {
        f2v xl[H2], wv[H2];
        lds_vec<RM>(xsl + l * V, lane, xl);
        lds_vec<RM>(sw + l * V, lane, wv);
        f2v d2 = f2v{0.f, 0.f};
#pragma unroll
        for (int h = 0; h < H2; ++h) d2 += gr[h] * xl[h];
        const float gx = wave_sum_dpp(d2[0] + d2[1]);
        const f2v gxv = f2v{gx, gx}, s1 = f2v{1.f + sl[l], 1.f + sl[l]};
#pragma unroll
        for (int h = 0; h < H2; ++h) {
          dba[l][h] += gr[h];
          dwa[l][h] += gxv * xl[h];
          gr[h] = gr[h] * s1 + gxv * wv[h];
        }
      }
      // dx0 = cross part + deep part -> embedding grads (or the total row,
      // for the deterministic embed_bwd.hip)
      if (p.dx0_tot) {   // table-major: table t's [B][w_t] block at B * off_t
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          const int t = m.tab[r];
          if (t >= 0)
            p.dx0_tot[B * tl.off[t] + b * tl.width[t] + m.col[r]] = gr[r >> 1][r & 1] + dd[u][r];
        }
        continue;
      }
      const int* ids_s = ids + s * g.n_tab;
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        const int t = m.tab[r];
        const float v = gr[r >> 1][r & 1] + dd[u][r];
        if constexpr (!(GC_LAB_MODE & 8))
          if (t >= 0) atomicAdd(tl.grad[t] + (int64_t)ids_s[t] * tl.width[t] + m.col[r], v);
      }
    }
  }
  // block-level partial: the 4 waves add into LDS in fixed wave order
  // (deterministic), then one coalesced store per block
  const int stride = (2 * L + 1) * D + 1;
  for (int ww = 0; ww < WPB; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        const int e = lane + WAVE * r;
        if (e >= D) continue;
#pragma unroll
        for (int l = 0; l < L; ++l) {
          red[l * D + e] = (ww ? red[l * D + e] : 0.f) + dwa[l][r >> 1][r & 1];
          red[(L + l) * D + e] = (ww ? red[(L + l) * D + e] : 0.f) + dba[l][r >> 1][r & 1];
        }
        red[2 * L * D + e] = (ww ? red[2 * L * D + e] : 0.f) + dwfa[r >> 1][r & 1];
      }
      if (lane == 0) red[(2 * L + 1) * D] = (ww ? red[(2 * L + 1) * D] : 0.f) + dbf;
    }
    __syncthreads();
  }
  float* mp = part + (int64_t)blockIdx.x * stride;
  for (int i = threadIdx.x; i < stride; i += NT) mp[i] = red[i];
}

// ----------------------------------------------- backward, 16-byte lanes
// Same chunk map and wave-owned id pipeline as gather_cross_v4_kernel.  Per
// tile a wave issues the x0 gathers and dx0_deep row loads of its SPW samples
// together, then per sample recomputes the cross stack (x_0..x_{L-1} kept in
// registers), runs its backward, accumulates dw_l / db_l / dw_f / db_f in
// registers, and scatter-adds dx0 = dx0_cross + dx0_deep into the dense
// embedding grads (fp32 no-return atomics, 4 per chunk).  Block partials are
// combined in fixed wave order (deterministic) for cross_reduce_kernel.
template <int R4, int L, int SPW>
__global__ __launch_bounds__(NT, 2) void cross_bwd_v4_kernel(GatherDesc g, CrossBwdParams p,
                                                           const int64_t* user,
                                                           const int64_t* item,
                                                           const int64_t* cat, const float* num,
                                                           const float* dz, int64_t B,
                                                           const float* dx0_deep, int ld_dx,
                                                           float* part) {
  constexpr int C = R4 * WAVE, LL = L > 0 ? L : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  const int D = g.D, nt = g.n_tab;
  v4f* sw = reinterpret_cast<v4f*>(smem);   // [L][C]
  v4f* sb = sw + L * C;                     // [L][C]
  v4f* swf = sb + L * C;                    // [C]
  float* red = reinterpret_cast<float*>(swf + C);   // [(2L+1)D+1] block partial
  // element maps of the dword layout used by the gradient scatter (e < 4C):
  // egrad[e] = grad row-0 address of element e, estride[e] = its row stride,
  // etab[e] = table index (-1: not a table element)
  float** egrad = reinterpret_cast<float**>(red + ((((2 * L + 1) * D + 1) + 3) & ~3));
  int* estride = reinterpret_cast<int*>(egrad + 4 * C);
  int* etab = estride + 4 * C;
  // per-wave dword image of the dx0 row being scattered
  v4f* wrow = reinterpret_cast<v4f*>(etab + 4 * C) + (threadIdx.x >> 6) * C;
  for (int i = threadIdx.x; i < (2 * L + 1) * C * 4; i += NT) {
    const int l = i / (C * 4), e = i % (C * 4);
    float v = 0.f;
    if (e < D) v = l < L ? p.cp.w[l][e] : l < 2 * L ? p.cp.b[l - L][e] : p.cp.wf_cross[e];
    smem[i] = v;
  }
  fill_tab_lds(g, tl, p.emb_grad);
  __syncthreads();
  for (int e = threadIdx.x; e < 4 * C; e += NT) {
    int t = -1;
    for (int q = 0; q < nt; ++q)
      if (e < D && e >= tl.off[q] && e < tl.off[q] + tl.width[q]) t = q;
    etab[e] = t;
    egrad[e] = t >= 0 ? tl.grad[t] + (e - tl.off[t]) : nullptr;
    estride[e] = t >= 0 ? tl.width[t] : 0;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* base[R4];
  int stride[R4], tab[R4];
#pragma unroll
  for (int r = 0; r < R4; ++r) {
    const int e = 4 * (lane + WAVE * r);
    int t = NO_ELEM, col = 0;
    if (e < D) {
      t = NUM_TAB;
      col = e - (D - g.n_num);
      for (int q = 0; q < nt; ++q)
        if (e >= tl.off[q] && e < tl.off[q] + tl.width[q]) { t = q; col = e - tl.off[q]; }
    }
    tab[r] = t;
    base[r] = t >= 0 ? tl.tab[t] + col : (t == NUM_TAB ? num + col : tl.tab[0]);
    stride[r] = t >= 0 ? tl.width[t] : (t == NUM_TAB ? g.n_num : 0);
  }
  const int ju = lane / nt, jt = lane % nt;
  const int64_t jrows = tl.rows[jt];
  auto load_ids = [&](int64_t b0) {
    const int64_t b = b0 + ju;
    const bool ok = ju < SPW && b < B;
    const int64_t bc = ok ? b : 0;
    const int64_t* src = jt == 0 ? user + bc : jt == 1 ? item + bc : cat + bc * (nt - 2) + (jt - 2);
    int64_t raw = ok ? *src : 0;
    raw = raw < 0 ? 0 : (raw >= jrows ? jrows - 1 : raw);
    return (int)raw;
  };

  v4f dwa[LL][R4], dba[LL][R4], dwfa[R4];
  float dbf = 0.f;
#pragma unroll
  for (int r = 0; r < R4; ++r) {
    dwfa[r] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int l = 0; l < LL; ++l) dwa[l][r] = dba[l][r] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  const int64_t ntiles = (B + SPW - 1) / SPW;
  const int64_t wave_id = (int64_t)blockIdx.x * WPB + w;
  const int64_t n_waves = (int64_t)gridDim.x * WPB;
  int idc = wave_id < ntiles ? load_ids(wave_id * SPW) : 0;
  for (int64_t tile = wave_id; tile < ntiles; tile += n_waves) {
    const int64_t b0 = tile * SPW;
    v4f x[SPW][R4], dd[SPW][R4];
    float dzv[SPW];
    const int idc_u = idc;   // this tile's ids (idc is refilled with the next tile's below)
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int64_t bc = b0 + u < B ? b0 + u : B - 1;
#pragma unroll
      for (int r = 0; r < R4; ++r) {
        const int t = tab[r];
        const int id = __builtin_amdgcn_ds_bpermute((u * nt + (t >= 0 ? t : 0)) << 2, idc_u);
        const int64_t row = t >= 0 ? (int64_t)id : (t == NUM_TAB ? bc : 0);
        x[u][r] = *reinterpret_cast<const v4f*>(base[r] + row * stride[r]);
        const int e = 4 * (lane + WAVE * r);
        dd[u][r] = *reinterpret_cast<const v4f*>(dx0_deep + bc * ld_dx + (e < ld_dx ? e : 0));
      }
      dzv[u] = dz[bc];
    }
    if (tile + n_waves < ntiles) idc = load_ids((tile + n_waves) * SPW);
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      if (b0 + u >= B) break;
      v4f xs[LL][R4], xc[R4];
      float sl[LL];
#pragma unroll
      for (int r = 0; r < R4; ++r)
        xc[r] = tab[r] == NO_ELEM ? v4f{0.f, 0.f, 0.f, 0.f} : x[u][r];
#pragma unroll
      for (int l = 0; l < L; ++l) {
        float d = 0.f;
#pragma unroll
        for (int r = 0; r < R4; ++r) {
          xs[l][r] = xc[r];
          d += dot4(xc[r], sw[l * C + lane + WAVE * r]);
        }
        sl[l] = wave_sum_dpp(d);
#pragma unroll
        for (int r = 0; r < R4; ++r) xc[r] = (xc[r] + xc[r] * sl[l]) + sb[l * C + lane + WAVE * r];
      }
      const float dzb = dzv[u];
      dbf += dzb;
      v4f gr[R4];
#pragma unroll
      for (int r = 0; r < R4; ++r) {
        gr[r] = dzb * swf[lane + WAVE * r];
        dwfa[r] += dzb * xc[r];
      }
#pragma unroll
      for (int l = L - 1; l >= 0; --l) {
        float d = 0.f;
#pragma unroll
        for (int r = 0; r < R4; ++r) d += dot4(gr[r], xs[l][r]);
        const float gx = wave_sum_dpp(d), s1 = 1.f + sl[l];
#pragma unroll
        for (int r = 0; r < R4; ++r) {
          dba[l][r] += gr[r];
          dwa[l][r] += gx * xs[l][r];
          gr[r] = gr[r] * s1 + gx * sw[l * C + lane + WAVE * r];
        }
      }
      // dx0 = cross part + deep part -> dense embedding grads.  The row is
      // re-laid out through this wave's LDS image into one dword per lane
      // (element e = lane + 64 q), so each atomic wave-instruction adds two
      // contiguous 128-B row segments (the full-rate shape for memory-side
      // float atomics, MI355X_MICROARCH.md "Global float atomics").
      if (p.dx0_tot) {   // total dx0 for embed_bwd.hip, table-major ([B][w_t] per table)
        const int64_t b = b0 + u;
#pragma unroll
        for (int r = 0; r < R4; ++r) {
          const int t = tab[r];
          if (t >= 0) {
            const int col = 4 * (lane + WAVE * r) - tl.off[t];
            *reinterpret_cast<v4f*>(p.dx0_tot + B * tl.off[t] + b * tl.width[t] + col) =
                gr[r] + dd[u][r];
          }
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < R4; ++r) wrow[lane + WAVE * r] = gr[r] + dd[u][r];
      const float* wf1 = reinterpret_cast<const float*>(wrow);
#pragma unroll
      for (int q = 0; q < 4 * R4; ++q) {
        const int e = lane + WAVE * q;
        const int t = etab[e];
        const int id = __builtin_amdgcn_ds_bpermute((u * nt + (t >= 0 ? t : 0)) << 2, idc_u);
        if (t < 0 || (GC_LAB_MODE & 8)) continue;
        atomicAdd(egrad[e] + (int64_t)id * estride[e], wf1[e]);
      }
    }
  }
  // block partial, waves added in fixed order
  const int stride_p = (2 * L + 1) * D + 1;
  for (int ww = 0; ww < WPB; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int r = 0; r < R4; ++r) {
        const int e = 4 * (lane + WAVE * r);
        if (e >= D) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
          for (int l = 0; l < L; ++l) {
            red[l * D + e + k] = (ww ? red[l * D + e + k] : 0.f) + dwa[l][r][k];
            red[(L + l) * D + e + k] = (ww ? red[(L + l) * D + e + k] : 0.f) + dba[l][r][k];
          }
          red[2 * L * D + e + k] = (ww ? red[2 * L * D + e + k] : 0.f) + dwfa[r][k];
        }
      }
      if (lane == 0) red[(2 * L + 1) * D] = (ww ? red[(2 * L + 1) * D] : 0.f) + dbf;
    }
    __syncthreads();
  }
  float* mp = part + (int64_t)blockIdx.x * stride_p;
  for (int i = threadIdx.x; i < stride_p; i += NT) mp[i] = red[i];
}

// Reduce per-block partials -> grads.  Block = 64 columns x 4 partial lanes
// over a range of partial rows (RED_G ranges in blockIdx.y), fp32 block sums
// to cred2 [RED_G][stride], and the last arriver of each column group adds the
// RED_G sums in fixed order and writes the gradients.
__global__ __launch_bounds__(NT) void cross_reduce_kernel(const float* part, int nb, int D, int L,
                                                          CrossBwdParams p, float* red2,
                                                          int* counters, int accumulate) {
  __shared__ float red[4 * 64 + 1];
  int* flag = reinterpret_cast<int*>(&red[4 * 64]);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int stride = (2 * L + 1) * D + 1;
  const int i = blockIdx.x * 64 + tx;
  const int g = blockIdx.y;
  const int per = (nb + RED_G - 1) / RED_G;
  const int w0 = g * per, w1 = min(nb, w0 + per);
  const __amdgpu_buffer_rsrc_t pr = buf_rsrc(part, (int64_t)nb * stride * 4);
  constexpr int U = 8;
  float s = 0.f;
  for (int wr = w0 + ty; wr < w1; wr += 4 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ww = wr + 4 * u;
      const bool ok = i < stride && ww < w1;
      v[u] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(pr, ok ? (ww * stride + i) * 4 : OOR, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  red[ty * 64 + tx] = s;
  __syncthreads();
  if (ty == 0 && i < stride)
    red2[(int64_t)g * stride + i] = ((red[tx] + red[64 + tx]) + red[128 + tx]) + red[192 + tx];
  if (!last_arriver(&counters[blockIdx.x], RED_G, flag)) return;
  if (ty != 0 || i >= stride) return;
  const __amdgpu_buffer_rsrc_t rr = buf_rsrc(red2, (int64_t)RED_G * stride * 4);
  float v[RED_G];
#pragma unroll
  for (int q = 0; q < RED_G; ++q)
    v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, (q * stride + i) * 4, 0, 0));
  float t = 0.f;
#pragma unroll
  for (int q = 0; q < RED_G; ++q) t += v[q];
  float* dst;
  if (i < L * D) dst = p.dw[i / D] + i % D;
  else if (i < 2 * L * D) dst = p.db[(i - L * D) / D] + (i - L * D) % D;
  else if (i < stride - 1) dst = p.dwf_cross + (i - 2 * L * D);
  else dst = p.dbf;
  *dst = accumulate ? *dst + t : t;
}

// -------------------------------------------------------------- launchers
constexpr int FWD_SPW = 4;   // samples per wave per tile (forward)
constexpr int BWD_SPW = 1;   // (backward: 2 waves/SIMD need the registers)

template <typename T, int RM>
dcnr_status launch_fwd(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                       const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                       void* x0, int ldx, float* zc, int* err, int check, hipStream_t s,
                       float* cross = nullptr, int ldc = 0) {
  constexpr int S = FWD_SPW * WPB;
  size_t lds = (size_t)(((2 * cp.L + 1) * g.D + S * g.n_tab + 3) & ~3) * sizeof(float) +
               (size_t)WPB * RM * WAVE * sizeof(bf16);
  int64_t blocks = std::min<int64_t>(cdiv(B, S), 256 * 8);
  hipLaunchKernelGGL((gather_cross_fwd_kernel<T, RM, FWD_SPW>), dim3((unsigned)blocks), dim3(NT),
                     lds, s, g, cp, user, item, cat, num, B, (T*)x0, ldx, zc, err, check, cross, ldc);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

#ifndef GC_V4_SPW
#define GC_V4_SPW 4
#endif
#ifndef GC_V4_WAVES
#define GC_V4_WAVES 3072
#endif

template <int R4, int X0BF16>
dcnr_status launch_v4(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                      const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                      const GcOut& o, int* err, int check, hipStream_t s) {
  constexpr int SPW = GC_V4_SPW;
  const size_t lds = (size_t)(2 * cp.L + 1) * R4 * WAVE * 16;
  // about GC_V4_WAVES waves (measured best: ~3 per SIMD resident at once),
  // every wave taking the same number of tiles
  const int64_t ntiles = cdiv(B, SPW);
  const int64_t waves = cdiv(ntiles, cdiv(ntiles, GC_V4_WAVES));
  const unsigned blocks = (unsigned)cdiv(waves, WPB);
  if (SPW * g.n_tab <= 64)
    hipLaunchKernelGGL((gather_cross_v4_kernel<R4, SPW, 1, X0BF16>), dim3(blocks), dim3(NT), lds, s,
                       g, cp, user, item, cat, num, B, o, err, check);
  else
    hipLaunchKernelGGL((gather_cross_v4_kernel<R4, SPW, 2, X0BF16>), dim3(blocks), dim3(NT), lds, s,
                       g, cp, user, item, cat, num, B, o, err, check);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

// The 16-byte-lane kernel applies: widths, n_num, offsets 4-aligned, every
// pointer 16-B aligned, D <= 512, and the id map fits two registers.
bool v4_ok(const GatherDesc& g, const float* num, const GcOut& o) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (g.D > 2 * 4 * WAVE || g.n_num % 4 || g.n_tab * GC_V4_SPW > 128) return false;
  if (g.n_num && !al(num)) return false;
  for (int t = 0; t < g.n_tab; ++t)
    if (g.width[t] % 4 || g.off[t] % 4 || !al(g.tab[t])) return false;
  if (o.cross && (o.ld_cross % 4 || !al(o.cross))) return false;
  if (o.x0 && (o.ld_x0 % 4 || !al(o.x0))) return false;
  return true;
}

template <int RM, int L>
dcnr_status launch_bwd(const GatherDesc& g, const CrossBwdParams& p, const int64_t* user,
                       const int64_t* item, const int64_t* cat, const float* num, const float* dz,
                       int64_t B, const float* dx0, int ld_dx, float* part, int64_t nb,
                       hipStream_t s) {
  constexpr int S = BWD_SPW * WPB;
  size_t lds = (size_t)((2 * L + 1) * RM * WAVE + (((2 * L + 1) * g.D + 1 + 3) & ~3)) * sizeof(float) +
               (size_t)((S * g.n_tab + 3) & ~3) * sizeof(int) +
               (size_t)WPB * (L > 0 ? L : 1) * RM * WAVE * sizeof(float);
  static size_t attr_lds = 0;   // raise the dynamic-LDS limit once per size class
  if (lds > 64 * 1024 && lds > attr_lds) {
    DCNR_HIP(hipFuncSetAttribute((const void*)cross_bwd_kernel<RM, L, BWD_SPW>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_lds = lds;
  }
  hipLaunchKernelGGL((cross_bwd_kernel<RM, L, BWD_SPW>), dim3((unsigned)nb), dim3(NT), lds, s, g,
                     p, user, item, cat, num, dz, B, dx0, ld_dx, part);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

#ifndef GC_V4B_SPW
#define GC_V4B_SPW 2
#endif
#ifndef GC_V4B_WAVES
#define GC_V4B_WAVES 3072
#endif

template <int R4, int L>
dcnr_status launch_bwd_v4(const GatherDesc& g, const CrossBwdParams& p, const int64_t* user,
                          const int64_t* item, const int64_t* cat, const float* num,
                          const float* dz, int64_t B, const float* dx0, int ld_dx, float* part,
                          int64_t* nb_out, hipStream_t s) {
  constexpr int SPW = GC_V4B_SPW;
  const size_t lds = (size_t)(2 * L + 1) * R4 * WAVE * 16 +
                     (size_t)((((2 * L + 1) * g.D + 1) + 3) & ~3) * sizeof(float) +
                     (size_t)R4 * WAVE * 4 * (8 + 4 + 4) + (size_t)WPB * R4 * WAVE * 16;
  const int64_t ntiles = cdiv(B, SPW);
  const int64_t waves = cdiv(ntiles, cdiv(ntiles, GC_V4B_WAVES));
  const int64_t nb = std::min<int64_t>(cdiv(waves, WPB), BWD_BLOCKS);
  static size_t attr_lds = 0;
  if (lds > 64 * 1024 && lds > attr_lds) {
    DCNR_HIP(hipFuncSetAttribute((const void*)cross_bwd_v4_kernel<R4, L, SPW>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_lds = lds;
  }
  hipLaunchKernelGGL((cross_bwd_v4_kernel<R4, L, SPW>), dim3((unsigned)nb), dim3(NT), lds, s, g, p,
                     user, item, cat, num, dz, B, dx0, ld_dx, part);
  DCNR_LAUNCH_CHECK();
  *nb_out = nb;
  return DCNR_OK;
}

template <int R4>
dcnr_status dispatch_bwd_v4(int L, const GatherDesc& g, const CrossBwdParams& p,
                            const int64_t* user, const int64_t* item, const int64_t* cat,
                            const float* num, const float* dz, int64_t B, const float* dx0,
                            int ld_dx, float* part, int64_t* nb, hipStream_t s) {
  switch (L) {
#define CASE(n) \
  case n: return launch_bwd_v4<R4, n>(g, p, user, item, cat, num, dz, B, dx0, ld_dx, part, nb, s);
    CASE(0) CASE(1) CASE(2) CASE(3) CASE(4)
#undef CASE
  }
  return DCNR_UNSUPPORTED_SHAPE;
}

template <int RM>
dcnr_status dispatch_bwd_L(int L, const GatherDesc& g, const CrossBwdParams& p,
                           const int64_t* user, const int64_t* item, const int64_t* cat,
                           const float* num, const float* dz, int64_t B, const float* dx0,
                           int ld_dx, float* part, int64_t nb, hipStream_t s) {
  switch (L) {
#define CASE(n) \
  case n: return launch_bwd<RM, n>(g, p, user, item, cat, num, dz, B, dx0, ld_dx, part, nb, s);
    CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7)
#undef CASE
  }
  set_error("cross: n_cross_layers=%d unsupported (max 7)", L);
  return DCNR_UNSUPPORTED_SHAPE;
}

int64_t bwd_blocks(int64_t B) { return std::max<int64_t>(1, std::min<int64_t>(cdiv(B, BWD_SPW * WPB), BWD_BLOCKS)); }

}  // namespace

size_t cross_bwd_part_elems(int D, int L) { return (size_t)BWD_BLOCKS * ((2 * L + 1) * D + 1); }
size_t cross_red2_elems(int D, int L) { return (size_t)RED_G * ((2 * L + 1) * D + 1); }
int cross_red_groups(int D, int L) { return (int)cdiv((2 * L + 1) * D + 1, 64); }

dcnr_status gather_cross_fwd(int precision, const GatherDesc& g, const CrossParams& cp,
                             const int64_t* user, const int64_t* item, const int64_t* cat,
                             const float* num, int64_t B, void* x0, int ldx, float* zc, int* err,
                             int check, hipStream_t s) {
  if (B <= 0) return DCNR_OK;
  if (g.D > 16 * WAVE || cp.L > 8 || g.n_tab > MAX_TABLES) {
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

dcnr_status gather_cross_out(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                             const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                             const GcOut& o, int x0_bf16, int* err, int check, hipStream_t s) {
  if (B <= 0) return DCNR_OK;
  if (cp.L > 8 || g.n_tab > MAX_TABLES) {
    set_error("gather: unsupported n_cross=%d / tables=%d", cp.L, g.n_tab);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (!v4_ok(g, num, o)) {   // the general (4-byte lane) kernel
    if (g.D > 16 * WAVE || (o.x0 && o.ld_x0 > 16 * WAVE) || (o.cross && o.ld_cross > 16 * WAVE)) {
      set_error("gather: unsupported D=%d", g.D);
      return DCNR_UNSUPPORTED_SHAPE;
    }
    const bool small = g.D <= 8 * WAVE && (!o.x0 || o.ld_x0 <= 8 * WAVE) &&
                       (!o.cross || o.ld_cross <= 8 * WAVE);
    if (x0_bf16)
      return small ? launch_fwd<bf16, 8>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc, err,
                                         check, s, o.cross, o.ld_cross)
                   : launch_fwd<bf16, 16>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc,
                                          err, check, s, o.cross, o.ld_cross);
    return small ? launch_fwd<float, 8>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc, err,
                                        check, s, o.cross, o.ld_cross)
                 : launch_fwd<float, 16>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc, err,
                                         check, s, o.cross, o.ld_cross);
  }
  const bool r1 = g.D <= 4 * WAVE && (!o.x0 || o.ld_x0 <= 4 * WAVE) &&
                  (!o.cross || o.ld_cross <= 4 * WAVE);
  if (x0_bf16)
    return r1 ? launch_v4<1, 1>(g, cp, user, item, cat, num, B, o, err, check, s)
              : launch_v4<2, 1>(g, cp, user, item, cat, num, B, o, err, check, s);
  return r1 ? launch_v4<1, 0>(g, cp, user, item, cat, num, B, o, err, check, s)
            : launch_v4<2, 0>(g, cp, user, item, cat, num, B, o, err, check, s);
}

dcnr_status cross_bwd_scatter(const GatherDesc& g, const CrossBwdParams& p, const int64_t* user,
                              const int64_t* item, const int64_t* cat, const float* num,
                              const float* dz, int64_t B, const float* dx0_deep, int ld_dx,
                              const CrossBwdScratch& ws, int accumulate, hipStream_t s) {
  const int L = p.cp.L, D = g.D;
  if (ws.part_elems < cross_bwd_part_elems(D, L) || ws.red2_elems < cross_red2_elems(D, L) ||
      ws.n_counters < cross_red_groups(D, L)) {
    set_error("cross_bwd: scratch too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  if (D > 16 * WAVE) {
    set_error("cross_bwd: D=%d unsupported", D);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  int64_t nb = bwd_blocks(B);
  dcnr_status st;
  const GcOut chk{nullptr, const_cast<float*>(dx0_deep), nullptr, 0, ld_dx};
  const bool v4 = L <= 4 && g.n_tab * GC_V4B_SPW <= 64 && v4_ok(g, num, chk);
  if (v4)
    st = D <= 4 * WAVE && ld_dx <= 4 * WAVE
             ? dispatch_bwd_v4<1>(L, g, p, user, item, cat, num, dz, B, dx0_deep, ld_dx, ws.part,
                                  &nb, s)
             : dispatch_bwd_v4<2>(L, g, p, user, item, cat, num, dz, B, dx0_deep, ld_dx, ws.part,
                                  &nb, s);
  else
    st = D <= 8 * WAVE
                       ? dispatch_bwd_L<8>(L, g, p, user, item, cat, num, dz, B, dx0_deep, ld_dx,
                                           ws.part, nb, s)
                       : dispatch_bwd_L<16>(L, g, p, user, item, cat, num, dz, B, dx0_deep, ld_dx,
                                            ws.part, nb, s);
  if (st != DCNR_OK) return st;
  hipLaunchKernelGGL(cross_reduce_kernel, dim3((unsigned)cross_red_groups(D, L), RED_G), dim3(NT),
                     0, s, ws.part, (int)nb, D, L, p, ws.red2, ws.counters, accumulate);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}


}  // namespace dcnr
