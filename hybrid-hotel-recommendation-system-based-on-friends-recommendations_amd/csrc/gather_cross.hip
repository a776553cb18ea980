// Embedding gathers + x0 assembly + the cross stack, forward (gfx950, 64-lane
// waves).  The backward lives in cross_bwd.hip (low-rank form, from the
// per-sample scalars this forward saves) and embed_bwd.hip (the dense
// embedding gradients).
//
// Forward  (DCN_RecSys.forward, train.py:156-159 and 167-168):
//   x0[b] = [U[u_b] | I[i_b] | C_0[c_b0] ... C_{K-1}[c_b,K-1] | num_b]   (bit-exact fp32 gather)
//   x_{l+1} = x_l + x_l * (x_l . w_l) + b_l                               (CrossLayer, train.py:96-99)
//   zc[b] = w_f[H:] . x_L       (the cross half of final_linear, train.py:169-170)
// The cross output itself is never written (except for dcnr_gather_cross):
// the head only needs its dot with w_f.  x0 is written once, in the deep
// tower's storage type (A operand of the initial Linear).  In train mode the
// forward also saves s_l = x_l . w_l, u_m = x_0 . w_m and u_f = x_0 . w_f[H:]
// per sample (2L+1 floats), all the cross backward needs.
//
// Latency structure (the gathers are dependent loads: id -> row): a block
// stages the ids of a tile of samples in LDS with coalesced loads, then each
// wave issues the row loads of several samples back to back (unconditional
// loads at clamped addresses, so no per-element branch serialises them)
// before computing any of them.
#include "dcnr_internal.h"

#include <cstring>

namespace dcnr {
namespace {

constexpr int NT = 256;
constexpr int WPB = NT / WAVE;
constexpr int NUM_TAB = -1, NO_ELEM = -2;

struct TabLds {
  const float* tab[MAX_TABLES];
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

__device__ __forceinline__ void fill_tab_lds(const GatherDesc& g, TabLds& tl) {
  for (int i = threadIdx.x; i < g.n_tab; i += NT) {
    tl.tab[i] = g.tab[i];
    tl.rows[i] = (int)g.rows[i];
    tl.width[i] = g.width[i];
    tl.off[i] = g.off[i];
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
                                                               int check, float* cross, int ldc,
                                                               float* sc) {
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
  fill_tab_lds(g, tl);
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
      load_row<RM>(m, ids + s * g.n_tab, b < B ? b : B - 1, x[u]);
    }
    // x0 in the deep tower's storage type.  bf16: staged through this wave's
    // LDS row so every lane stores 16 contiguous bytes (8 columns)
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int64_t b = b0 + w * SPW + u;
      if (x0 == nullptr) continue;
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
    // the backward's per-sample scalars u_m = x_0 . w_m (m >= 1; u_0 = s_0)
    // and u_f = x_0 . w_f[H:] (the low-rank cross backward, cross_bwd.hip)
    const int nsc = 2 * L + 1;
    if (sc) {
      for (int m = L > 0 ? 1 : 0; m <= L; ++m) {
        const float* wm = m < L ? sw + m * D : swf;
        float d[SPW], us[SPW];
#pragma unroll
        for (int u = 0; u < SPW; ++u) {
          d[u] = 0.f;
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            const int e = lane + WAVE * r;
            if (e < D) d[u] += x[u][r] * wm[e];
          }
        }
        wave_sum4(d[0], d[1], d[2], d[3], us[0], us[1], us[2], us[3]);
        const int64_t b = b0 + w * SPW + lane;
        if (lane < SPW && b < B)
          sc[b * nsc + L + m] = lane == 0 ? us[0] : lane == 1 ? us[1] : lane == 2 ? us[2] : us[3];
      }
    }
    // cross stack: the SPW (=4) samples' dot products are reduced together
    {
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
        if (sc) {
          const int64_t b = b0 + w * SPW + lane;
          if (lane < SPW && b < B) {
            const float sv = lane == 0 ? sl[0] : lane == 1 ? sl[1] : lane == 2 ? sl[2] : sl[3];
            sc[b * nsc + l] = sv;
            if (l == 0) sc[b * nsc + L] = sv;   // u_0 = s_0
          }
        }
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
  fill_tab_lds(g, tl);
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
    // the backward's per-sample scalars u_m = x_0 . w_m (m >= 1; u_0 = s_0)
    // and u_f = x_0 . w_f[H:] (the low-rank cross backward, cross_bwd.hip)
    const int nsc = 2 * L + 1;
    if (out.sc) {
      for (int m = L > 0 ? 1 : 0; m <= L; ++m) {
        v4f wv[R4];
#pragma unroll
        for (int r = 0; r < R4; ++r) wv[r] = m < L ? sw[m * C + lane + WAVE * r] : swf[lane + WAVE * r];
#pragma unroll
        for (int u0 = 0; u0 < SPW; u0 += 4) {
          float d[4], us[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            d[k] = 0.f;
#pragma unroll
            for (int r = 0; r < R4; ++r) d[k] += dot4(x[u0 + k][r], wv[r]);
          }
          wave_sum4(d[0], d[1], d[2], d[3], us[0], us[1], us[2], us[3]);
          if (lane < 4 && b0 + u0 + lane < B)
            out.sc[(b0 + u0 + lane) * nsc + L + m] =
                lane == 0 ? us[0] : lane == 1 ? us[1] : lane == 2 ? us[2] : us[3];
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
        if (out.sc && lane < 4 && b0 + u0 + lane < B) {
          const float sv = lane == 0 ? s[0] : lane == 1 ? s[1] : lane == 2 ? s[2] : s[3];
          out.sc[(b0 + u0 + lane) * nsc + l] = sv;
          if (l == 0) out.sc[(b0 + u0 + lane) * nsc + L] = sv;   // u_0 = s_0
        }
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

// ------------------------------------------- low-rank front (train / eval)
// The deep forward never needs the cross output x_L itself, only zc = w_f[H:]
// . x_L (and in train mode the backward's scalars).  CrossLayer keeps every
// x_l in span{x_0, b_0 .. b_{l-1}} (x_{l+1} = (1 + s_l) x_l + b_l,
// train.py:96-99), so with x_l = a_l x_0 + sum_j e_lj b_j
//   s_l = x_l . w_l = a_l u_l + sum_{j<l} e_lj (b_j . w_l),     u_l = x_0 . w_l
//   a_{l+1} = (1 + s_l) a_l,  e_{l+1,j} = (1 + s_l) e_lj,  e_{l+1,l} = 1
//   zc = a_L u_f + sum_j e_Lj (b_j . w_f[H:]),                   u_f = x_0 . w_f[H:]
// -- the same algebra the low-rank backward (cross_bwd.hip) runs on.  Per
// sample: L + 1 dot products of the gathered x0 row (4 samples per wave
// reduction) and scalar arithmetic; no D-wide cross stack, no per-layer
// reduction of x_l.  The Gram terms b_j . w_m are computed per block, in a
// fixed order, from the parameters.  (fp32 throughout; it differs from the
// elementwise stack by rounding only: zc and the scalars are checked against
// fp64 in tests/test_stages_gpu.py and test_gather_cross_gpu.py.)
template <int R4, int SPW, int IDR, int X0BF16, int L>
__global__ __launch_bounds__(NT) void gather_lowrank_kernel(GatherDesc g, CrossParams cp,
                                                            const int64_t* user, const int64_t* item,
                                                            const int64_t* cat, const float* num,
                                                            int64_t B, GcOut out, int* err, int check) {
  static_assert(SPW % 4 == 0 && L >= 1 && L <= 4, "4 samples per reduction, 1..4 layers");
  constexpr int C = R4 * WAVE;       // float4 chunks per image
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ TabLds tl;
  __shared__ float gram[L][L + 1];   // b_j . w_m (m < L), b_j . w_f[H:] (m = L)
  const int D = g.D, nt = g.n_tab;
  v4f* sw = reinterpret_cast<v4f*>(smem);   // [L + 1][C]: w_0 .. w_{L-1}, w_f[H:] (0 past D)
  for (int i = threadIdx.x; i < (L + 1) * C * 4; i += NT) {
    const int l = i / (C * 4), e = i % (C * 4);
    smem[i] = e < D ? (l < L ? cp.w[l][e] : cp.wf_cross[e]) : 0.f;
  }
  fill_tab_lds(g, tl);
  // the Gram terms: one wave per term, lanes over D in order, a fixed tree
  for (int t = threadIdx.x >> 6; t < L * (L + 1); t += WPB) {
    const int j = t / (L + 1), m = t % (L + 1);
    const float* wm = m < L ? cp.w[m] : cp.wf_cross;
    float acc = 0.f;
    for (int e = threadIdx.x & 63; e < D; e += WAVE) acc = fmaf(cp.b[j][e], wm[e], acc);
    acc = wave_sum_dpp(acc);
    if ((threadIdx.x & 63) == 0) gram[j][m] = acc;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
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
  float G[L][L + 1];
#pragma unroll
  for (int j = 0; j < L; ++j)
#pragma unroll
    for (int m = 0; m <= L; ++m) G[j][m] = gram[j][m];
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

  constexpr int NSC = 2 * L + 1;
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
#pragma unroll
    for (int u0 = 0; u0 < SPW; u0 += 4) {
      // us[m][k]: x_0 . w_m (m < L), x_0 . w_f[H:] (m = L) of sample u0 + k
      float us[L + 1][4];
#pragma unroll
      for (int m = 0; m <= L; ++m) {
        v4f wv[R4];
#pragma unroll
        for (int r = 0; r < R4; ++r) wv[r] = sw[m * C + lane + WAVE * r];
        float d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[k] = 0.f;
#pragma unroll
          for (int r = 0; r < R4; ++r) d[k] += dot4(x[u0 + k][r], wv[r]);
        }
        wave_sum4(d[0], d[1], d[2], d[3], us[m][0], us[m][1], us[m][2], us[m][3]);
      }
      // the recurrence (wave-uniform scalars)
      float vals[4][NSC], zcv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 1.f, e[L];
#pragma unroll
        for (int l = 0; l < L; ++l) {
          float s = a * us[l][k];
#pragma unroll
          for (int j = 0; j < l; ++j) s = fmaf(e[j], G[j][l], s);
          vals[k][l] = s;
          vals[k][L + l] = us[l][k];
          const float f = 1.f + s;
          a *= f;
#pragma unroll
          for (int j = 0; j < l; ++j) e[j] *= f;
          e[l] = 1.f;
        }
        vals[k][2 * L] = us[L][k];
        float z = a * us[L][k];
#pragma unroll
        for (int j = 0; j < L; ++j) z = fmaf(e[j], G[j][L], z);
        zcv[k] = z;
      }
      if (out.zc) {
        float zl = zcv[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) zl = lane == k ? zcv[k] : zl;
        if (lane < 4 && b0 + u0 + lane < B) out.zc[b0 + u0 + lane] = zl;
      }
      if (out.sc && lane < 4 && b0 + u0 + lane < B) {   // lane k: sample u0 + k's NSC scalars
#pragma unroll
        for (int i = 0; i < NSC; ++i) {
          float v = vals[0][i];
#pragma unroll
          for (int k = 1; k < 4; ++k) v = lane == k ? vals[k][i] : v;
          out.sc[(b0 + u0 + lane) * NSC + i] = v;
        }
      }
    }
  }
}

// -------------------------------------------------------------- launchers
constexpr int FWD_SPW = 4;   // samples per wave per tile (forward)

template <typename T, int RM>
dcnr_status launch_fwd(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                       const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                       void* x0, int ldx, float* zc, int* err, int check, hipStream_t s,
                       float* cross = nullptr, int ldc = 0, float* sc = nullptr) {
  constexpr int S = FWD_SPW * WPB;
  size_t lds = (size_t)(((2 * cp.L + 1) * g.D + S * g.n_tab + 3) & ~3) * sizeof(float) +
               (size_t)WPB * RM * WAVE * sizeof(bf16);
  int64_t blocks = std::min<int64_t>(cdiv(B, S), 256 * 8);
  hipLaunchKernelGGL((gather_cross_fwd_kernel<T, RM, FWD_SPW>), dim3((unsigned)blocks), dim3(NT),
                     lds, s, g, cp, user, item, cat, num, B, (T*)x0, ldx, zc, err, check, cross, ldc,
                     sc);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

constexpr int GC_V4_SPW = 4;   // samples per wave-tile
// waves per launch (measured, same box, tools/ab_variants.sh): writing x0
// (train / eval forward) 4096 -- every wave resident at 4 per SIMD (104
// VGPRs) -- (round 4, tools/gather_probe.py, profiles/lab/r04q_gather_waves_ab.txt:
// train 84.0 vs 88.7 us, eval 61.8 vs 63.4 at 3072; 2560: 103.6 / 69.1;
// earlier: 2048 +20 %, 6144 +12 % kernel time); the gather + cross front
// alone (configs[1]) 2048 (+6 % pairs/s over 3072)
constexpr int GC_V4_WAVES = 4096, GC_V4_WAVES_NOX0 = 2048;

template <int R4, int X0BF16>
dcnr_status launch_v4(const GatherDesc& g, const CrossParams& cp, const int64_t* user,
                      const int64_t* item, const int64_t* cat, const float* num, int64_t B,
                      const GcOut& o, int* err, int check, hipStream_t s) {
  constexpr int SPW = GC_V4_SPW;
  const size_t lds = (size_t)(2 * cp.L + 1) * R4 * WAVE * 16;
  // about `target` waves (~2-3 per SIMD resident at once), every wave
  // taking the same number of tiles
  const int64_t ntiles = cdiv(B, SPW);
  const int64_t target = o.x0 ? GC_V4_WAVES : GC_V4_WAVES_NOX0;
  const int64_t waves = cdiv(ntiles, cdiv(ntiles, target));
  const unsigned blocks = (unsigned)cdiv(waves, WPB);
  if (o.x0 && !o.cross && cp.L >= 1 && cp.L <= 4) {   // the deep forward: the low-rank front
    const size_t lr_lds = (size_t)(cp.L + 1) * R4 * WAVE * 16;
    const bool i1 = SPW * g.n_tab <= 64;
#define DCNR_LR(LL)                                                                                    \
  if (cp.L == LL) {                                                                                    \
    if (i1)                                                                                            \
      hipLaunchKernelGGL((gather_lowrank_kernel<R4, SPW, 1, X0BF16, LL>), dim3(blocks), dim3(NT), lr_lds, \
                         s, g, cp, user, item, cat, num, B, o, err, check);                           \
    else                                                                                               \
      hipLaunchKernelGGL((gather_lowrank_kernel<R4, SPW, 2, X0BF16, LL>), dim3(blocks), dim3(NT), lr_lds, \
                         s, g, cp, user, item, cat, num, B, o, err, check);                           \
  }
    DCNR_LR(1) DCNR_LR(2) DCNR_LR(3) DCNR_LR(4)
#undef DCNR_LR
    DCNR_LAUNCH_CHECK();
    return DCNR_OK;
  }
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


}  // namespace


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
                                         check, s, o.cross, o.ld_cross, o.sc)
                   : launch_fwd<bf16, 16>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc,
                                          err, check, s, o.cross, o.ld_cross, o.sc);
    return small ? launch_fwd<float, 8>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc, err,
                                        check, s, o.cross, o.ld_cross, o.sc)
                 : launch_fwd<float, 16>(g, cp, user, item, cat, num, B, o.x0, o.ld_x0, o.zc, err,
                                         check, s, o.cross, o.ld_cross, o.sc);
  }
  const bool r1 = g.D <= 4 * WAVE && (!o.x0 || o.ld_x0 <= 4 * WAVE) &&
                  (!o.cross || o.ld_cross <= 4 * WAVE);
  if (x0_bf16)
    return r1 ? launch_v4<1, 1>(g, cp, user, item, cat, num, B, o, err, check, s)
              : launch_v4<2, 1>(g, cp, user, item, cat, num, B, o, err, check, s);
  return r1 ? launch_v4<1, 0>(g, cp, user, item, cat, num, B, o, err, check, s)
            : launch_v4<2, 0>(g, cp, user, item, cat, num, B, o, err, check, s);
}

}  // namespace dcnr
