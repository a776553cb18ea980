// Weight-resident streaming GEMM for the bf16 deep tower (gfx950):
//
//   C[M, N] = X[M, K] . W[N, K]^T  (+ bias | + residual),  K <= 512
//
// The deep tower's Linear layers (train.py:143,105,109) have a huge M (the
// batch, 131072) and a small N x K weight (<= 512 x 512): the problem is one
// pass over the activations.  Design:
//  * each workgroup keeps a 128-row slice of W resident in LDS for its whole
//    lifetime (128 x K bf16 <= 128 KiB, XOR-swizzled so the ds_read_b128
//    fragment reads are bank-conflict free) -- one barrier, at the start;
//  * each of the 4 waves owns 32 rows of every 128-row M-tile and loads its X
//    fragments straight from HBM into registers (the 16x16x32 B-operand
//    layout is 16 rows x 64 contiguous bytes per load), through a ring
//    DEPTH k-steps deep that runs continuously across the wave's M-tiles:
//    no LDS staging and no barrier in the main loop, counted vmcnt waits;
//  * workgroups are grouped so the N-slices of one M-tile run on one XCD at
//    the same time (blocks b, b+8, ... share an XCD's L2): X comes from HBM
//    once and is re-read from L2 by the other slices;
//  * v_mfma_f32_16x16x32_bf16 with W as the A operand and X as the B operand:
//    each lane accumulates 4 consecutive output columns of one row, so the
//    epilogue stores are 8-byte (bf16) / 16-byte (f32) row-contiguous;
//  * all global accesses go through range-checked buffer descriptors
//    (out-of-range loads read 0, stores are dropped): branch-free edges.
#include "dcnr_internal.h"

// tools/gemm_lab.hip rebuilds this file with NT_LAB_MODE bits set to time
// parts of the kernel in isolation (1: no C stores, 2: no X loads in the
// k-loop, 4: no MFMAs, 8: C stores into a 4096-row window, 16: X loads from a
// 4096-row window).  The library always builds mode 0.
#ifndef NT_LAB_MODE
#define NT_LAB_MODE 0
#endif

namespace dcnr {
namespace {

// NT_WAVES waves of NT_RB 16-row blocks each (tools/gemm_lab.hip sweeps both)
#ifndef NT_WAVES
#define NT_WAVES 8
#endif
#ifndef NT_RB
#define NT_RB 2
#endif
#ifndef NT_STORE_AUX
#define NT_STORE_AUX 0
#endif
#ifndef NT_EPI_SPREAD
#define NT_EPI_SPREAD 0
#endif
#ifndef NT_R_EARLY
#define NT_R_EARLY 0
#endif
#ifndef NT_DEPTH
#define NT_DEPTH 8
#endif
#ifndef NT_DEPTH_STATS
#define NT_DEPTH_STATS 4
#endif
#ifndef NT_WAVES_STATS
#define NT_WAVES_STATS 4
#endif
constexpr int RB = NT_RB, WROWS = 16 * RB, TN = 128, BK = 32;
// stats epilogues hold more live state: one wave per SIMD (512 registers)
//  * plain epilogues: 8 waves (2 per SIMD), ring depth 8;
//  * BIAS_STATS: 8 waves, ring depth 4 (registers for the per-tile partials);
//  * RESID_BN / DROP_BN: 4 waves (512 registers each) -- the mask/BN operands
//    and partials kept over all tiles.
template <int EPI> struct Geo {
  static constexpr bool HT = EPI == NT_EPI_RESID_BN || EPI == NT_EPI_DROP_BN;
  static constexpr int NWAVE = HT ? NT_WAVES_STATS : NT_WAVES;
  static constexpr int DEPTH = EPI == NT_EPI_BIAS_STATS ? NT_DEPTH_STATS : NT_DEPTH;
  static constexpr bool PERSIST = HT && NWAVE == 4;
  static constexpr int NT = 64 * NWAVE, TM = NWAVE * WROWS;
};
constexpr int TM_MIN = 64 * WROWS / 16;   // smallest TM of any epilogue (4 waves)

template <int KTP> struct NtCfg {
  static constexpr int WCH = KTP * (BK / 8);                 // 16-B chunks per W row
  static constexpr int DEPTH = KTP;   // (capped per epilogue by Geo::DEPTH)
  static constexpr int W_LDS = TN * WCH;                     // uint4 units
  static constexpr int BIAS_LDS = 3 * TN / 4;                // uint4 units (bias, mean, invstd)
  static constexpr size_t LDS_BYTES = (size_t)(W_LDS + BIAS_LDS) * 16;
};

template <int WCH>
__device__ __forceinline__ int w_slot(int row, int ch) { return row * WCH + (ch ^ (row & 15)); }


__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16 x = (bf16)a, y = (bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

// X fragments of one k-step for this wave: rows r0 + i*16 + (lane&15), k = kt*32 + 8*(lane>>4)
__device__ __forceinline__ void load_x(u32x4 (&f)[RB], __amdgpu_buffer_rsrc_t xr, int64_t ldx,
                                       int64_t M, int K, int64_t r0, int kt, int lane, bool valid) {
  const int k = kt * BK + 8 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    int64_t m = r0 + i * 16 + (lane & 15);
    if constexpr (NT_LAB_MODE & 16) m &= 4095;   // lab: X reads from a 4096-row window
    const bool ok = valid && m < M && k < K;
    f[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (int)((m * ldx + k) * 2) : OOR, 0, 0);
  }
}

// An epilogue operand tile (rows r0 + 16i + (lane&15), 128 columns from n0)
// loaded in the store layout: 16 B per lane, columns 16(2jp + (q&1)) +
// 8(q>>1) .. +7 -- 64 contiguous bytes per row and instruction.
__device__ __forceinline__ u32x4 load_epi1(__amdgpu_buffer_rsrc_t r, int64_t ld, int64_t r0, int i,
                                           int jp, int n0, int N, int64_t M, int lane) {
  const int q = lane >> 4;
  const int64_t m = r0 + i * 16 + (lane & 15);
  const int n = n0 + (2 * jp + (q & 1)) * 16 + (q >> 1) * 8;
  const bool ok = n < N && m < M;
  return __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (int)((m * ld + n) * 2) : OOR, 0, 0);
}
__device__ __forceinline__ void load_epi(u32x4 (&o)[RB][4], __amdgpu_buffer_rsrc_t r, int64_t ld,
                                         int64_t r0, int n0, int N, int64_t M, int lane) {
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) o[i][jp] = load_epi1(r, ld, r0, i, jp, n0, N, M, lane);
}
// store layout -> accumulator layout of fragments 2jp, 2jp+1 (columns
// 16j + 4q .. +3): the inverse of the epilogue's v_permlane16_swap (an involution)
__device__ __forceinline__ void to_acc_layout(const u32x4& L, u32x2 (&f)[2]) {
  auto a = __builtin_amdgcn_permlane16_swap(L[0], L[2], false, false);
  auto b = __builtin_amdgcn_permlane16_swap(L[1], L[3], false, false);
  f[0] = u32x2{a[0], b[0]};
  f[1] = u32x2{a[1], b[1]};
}

typedef float f2v __attribute__((ext_vector_type(2)));

// bf16 pair (low half = first) -> two floats
__device__ __forceinline__ f2v unpack2(uint32_t w) {
  return f2v{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}

// One reduce-scatter step over lane pairs (lane, partner(lane)) given by the
// DPP control: x[u] (u < H) becomes the pair-sum of x[u] (hi = false) or of
// x[u + H] (hi = true); partners have opposite `hi`.
template <int H, int CTRL>
__device__ __forceinline__ void bfly_step(float (&x)[64], bool hi) {
#pragma unroll
  for (int u = 0; u < H; ++u) {
    const float give = hi ? x[u] : x[u + H];
    const float keep = hi ? x[u + H] : x[u];
    x[u] = keep + dpp<CTRL>(give);
  }
}

// Reduce-scatter the 64 per-lane partials over the 16 lanes of a lane row
// (same columns, different rows): 4 DPP butterfly steps, each lane keeps half
// of what it holds (selected by one lane bit) and adds the partner's copy.
// Value index v = k*32 + j*4 + r; the lane's 4 results are added to tot.
__device__ __forceinline__ void stats_reduce(const f2v (&st)[2][8][2], float (&tot)[4], int lane) {
  float x[64];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) x[k * 32 + j * 4 + r] = st[k][j][r >> 1][r & 1];
  bfly_step<32, 0x141>(x, (lane & 4) != 0);   // partner lane^7, keep by bit 2
  bfly_step<16, 0x128>(x, (lane & 8) != 0);   // lane^8 (row_ror:8), bit 3
  bfly_step<8, 0xB1>(x, (lane & 1) != 0);     // lane^1, bit 0
  bfly_step<4, 0x4E>(x, (lane & 2) != 0);     // lane^2, bit 1
#pragma unroll
  for (int u = 0; u < 4; ++u) tot[u] += x[u];
}

template <int KTP, int EPI>
__global__ __launch_bounds__(Geo<EPI>::NT, 1) void gemm_nt_kernel(NtArgs a) {
  constexpr bool STATS = EPI >= NT_EPI_BIAS_STATS;
  constexpr int NT = Geo<EPI>::NT, TM = Geo<EPI>::TM, NWAVE = Geo<EPI>::NWAVE;
  constexpr bool PERSIST = Geo<EPI>::PERSIST;
  constexpr bool HAS_BIAS = EPI <= NT_EPI_BIAS_STATS;
  using C = NtCfg<KTP>;
  constexpr int DEPTH = KTP < Geo<EPI>::DEPTH ? KTP : Geo<EPI>::DEPTH;   // prefetch ring (k-steps)
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  uint4* Ws = lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nsl = a.nslices;
  const int bid = blockIdx.x;
  const int slice = (bid / 8) % nsl;
  const int group = (bid % 8) + 8 * (bid / (8 * nsl));
  const int groups = a.groups;
  const int n0 = slice * TN;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.X, (short)0, (int)(a.M * a.ldx * 2), 0x00020000);
  const int es = EPI == NT_EPI_F32 ? 4 : 2;
  const __amdgpu_buffer_rsrc_t cr =
      __builtin_amdgcn_make_buffer_rsrc(a.C, (short)0, (int)(a.M * a.ldc * es), 0x00020000);
  constexpr bool HAS_R = EPI == NT_EPI_RESID || EPI == NT_EPI_RESID_BN;
  constexpr bool HAS_HT = EPI == NT_EPI_RESID_BN || EPI == NT_EPI_DROP_BN;
  const __amdgpu_buffer_rsrc_t rr_ = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.R, (short)0, HAS_R ? (int)(a.M * a.ldr * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.H, (short)0, HAS_HT ? (int)(a.M * a.ldh * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.T, (short)0, HAS_HT ? (int)(a.M * a.ldt * 2) : 0, 0x00020000);
  float tot[4] = {0.f, 0.f, 0.f, 0.f};   // stats epilogues: this lane's share over all tiles
  // per-lane column partials [sum, sum2][fragment j][column pair]: per tile, or
  // (PERSIST, one wave per SIMD: registers to spare) over all of the WG's tiles
  f2v st[2][8][2];
  if constexpr (STATS && PERSIST) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 2; ++r) st[k][j][r] = f2v{0.f, 0.f};
  }

  // start the X stream before the W slice load so both are in flight
  u32x4 ring[DEPTH][RB];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    load_x(ring[d], xr, a.ldx, a.M, a.K, (int64_t)group * TM + wave * WROWS, d, lane,
           group < a.mtiles);

  // resident W slice (rows n0..n0+127, zero-padded beyond N and K)
  const int kch = a.K / 8;
  for (int c = tid; c < C::W_LDS; c += NT) {
    const int row = c / C::WCH, ch = c % C::WCH;
    const int n = n0 + row;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < a.N && ch < kch) v = *reinterpret_cast<const uint4*>(a.W + (int64_t)n * a.ldw + ch * 8);
    Ws[w_slot<C::WCH>(row, ch)] = v;
  }

  // bias (and BN mean / invstd) slices in LDS, read per tile in the
  // epilogue (registers go to the ring)
  float* bias_s = reinterpret_cast<float*>(lds + C::W_LDS);
  float* nmi_s = bias_s + TN;    // -mean * invstd
  float* istd_s = bias_s + 2 * TN;
  for (int c = tid; c < TN; c += NT) {
    const int n = n0 + c;
    bias_s[c] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
    if constexpr (HAS_HT) {
      nmi_s[c] = n < a.N ? -a.mean[n] * a.invstd[n] : 0.f;
      istd_s[c] = n < a.N ? a.invstd[n] : 0.f;
    }
  }
  __syncthreads();

  // W fragments of the current k-step (one buffer: each fragment is re-read
  // for the next k-step right after its two MFMAs have issued)
  bf16x8 wf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    wf[j] = __builtin_bit_cast(bf16x8, Ws[w_slot<C::WCH>(j * 16 + (lane & 15), lane >> 4)]);

  for (int64_t mt = group; mt < a.mtiles; mt += groups) {
    const int64_t r0 = mt * TM + wave * WROWS;
    // epilogue operands of this tile: residual, mask source, BN input
    u32x4 resid[RB][4], hv[RB][4], tv[RB][4];
#if NT_R_EARLY
    // (issued ahead of the k-loop's refills)
    if constexpr (HAS_R) load_epi(resid, rr_, a.ldr, r0, n0, a.N, a.M, lane);
#endif
    f32x4 acc[RB][8];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int kt = 0; kt < KTP; ++kt) {
      const int slot = kt % DEPTH;
      const int kn = (kt + 1) % KTP;   // next k-step (wraps to the next M-tile: W is tile-independent)
      bf16x8 xf[RB];
#pragma unroll
      for (int i = 0; i < RB; ++i) xf[i] = __builtin_bit_cast(bf16x8, ring[slot][i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int i = 0; i < RB; ++i)
          if constexpr (!(NT_LAB_MODE & 4))
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
          else
            acc[i][j][0] += (float)xf[i][j] + (float)wf[j][0];
        wf[j] = __builtin_bit_cast(bf16x8, Ws[w_slot<C::WCH>(j * 16 + (lane & 15), kn * 4 + (lane >> 4))]);
      }
#if NT_EPI_SPREAD
      // this tile's epilogue operands, spread evenly over the k-steps (a
      // steady trickle beside the ring refills instead of a burst at the end)
      if constexpr (HAS_R || HAS_HT) {
        constexpr int NOP = (HAS_R ? 1 : 0) + (HAS_HT ? 2 : 0), NL = NOP * RB * 4;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          if (l * KTP / NL != kt) continue;
          const int op = l / (RB * 4), i = (l / 4) % RB, jp = l % 4;
          const int which = HAS_R ? op : op + 1;   // 0: R, 1: H, 2: T
          if (which == 0) resid[i][jp] = load_epi1(rr_, a.ldr, r0, i, jp, n0, a.N, a.M, lane);
          else if (which == 1) hv[i][jp] = load_epi1(hr, a.ldh, r0, i, jp, n0, a.N, a.M, lane);
          else tv[i][jp] = load_epi1(tr, a.ldt, r0, i, jp, n0, a.N, a.M, lane);
        }
      }
#endif
      // refill the slot with the k-step DEPTH ahead (same or next M-tile)
      if constexpr (!(NT_LAB_MODE & 2)) {
        const int kd = kt + DEPTH;
        const int64_t mtn = mt + (kd >= KTP ? groups : 0);
        load_x(ring[slot], xr, a.ldx, a.M, a.K, mtn * TM + wave * WROWS, kd % KTP, lane,
               mtn < a.mtiles);
      }
      // pin the order: per j, RB MFMAs then the fragment's re-read
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, RB, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x020, RB, 0);    // VMEM read (ring refill)
      __builtin_amdgcn_sched_barrier(0);
    }

    // epilogue: lane holds C[m][n..n+3] of each (i, j), n = 16j + 4*(lane>>4).
    // bf16: fragments j and j+1 are exchanged between lane rows with
    // v_permlane16_swap so every lane stores 8 consecutive columns (16 B) and
    // each store instruction writes 64 contiguous bytes per output row.
    const int q = lane >> 4;
#if !NT_R_EARLY && !NT_EPI_SPREAD
    if constexpr (HAS_R) load_epi(resid, rr_, a.ldr, r0, n0, a.N, a.M, lane);
#endif
#if !NT_EPI_SPREAD
    if constexpr (HAS_HT) {
      load_epi(hv, hr, a.ldh, r0, n0, a.N, a.M, lane);
      load_epi(tv, tr, a.ldt, r0, n0, a.N, a.M, lane);
    }
#endif
    if constexpr (STATS && !PERSIST) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 2; ++r) st[k][j][r] = f2v{0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int64_t m = r0 + i * 16 + (lane & 15);
      const bool mok = m < a.M;
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        u32x2 o[2];
        u32x4 of[2];
        u32x2 rf[2], hf[2], tf[2];   // epilogue operands of fragments 2jp, 2jp+1
        if constexpr (HAS_R) to_acc_layout(resid[i][jp], rf);
        if constexpr (HAS_HT) {
          to_acc_layout(hv[i][jp], hf);
          to_acc_layout(tv[i][jp], tf);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * jp + h;
          // two column pairs (4q, 4q+1) and (4q+2, 4q+3) of fragment j
          f2v v[2] = {f2v{acc[i][j][0], acc[i][j][1]}, f2v{acc[i][j][2], acc[i][j][3]}};
          f2v bb[2];
          if constexpr (HAS_BIAS) {
            const float4 bj = *reinterpret_cast<const float4*>(bias_s + j * 16 + q * 4);
            bb[0] = f2v{bj.x, bj.y};
            bb[1] = f2v{bj.z, bj.w};
            v[0] += bb[0];
            v[1] += bb[1];
          }
          if constexpr (HAS_R) {
#pragma unroll
            for (int d = 0; d < 2; ++d) v[d] += unpack2(rf[h][d]);
          }
          if constexpr (EPI == NT_EPI_DROP_BN) {
            v[0] *= a.hscale;
            v[1] *= a.hscale;
          }
          o[h] = u32x2{pack2(v[0][0], v[0][1]), pack2(v[1][0], v[1][1])};
          of[h] = u32x4{__float_as_uint(v[0][0]), __float_as_uint(v[0][1]),
                        __float_as_uint(v[1][0]), __float_as_uint(v[1][1])};
          if constexpr (HAS_HT) {
            // RESID_BN: keep where h > 0 (bf16 bits: magnitude != 0, sign clear);
            // DROP_BN: keep where h != 0 (the saved dropout activation)
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              const uint32_t hw = hf[h][d];
              uint32_t keep = ((hw & 0x7fff7fffu) + 0x7fff7fffu) & 0x80008000u;
              if constexpr (EPI == NT_EPI_RESID_BN) keep &= ~hw;
              o[h][d] &= (keep >> 15) * 0xffffu;
            }
          }
          if constexpr (STATS) {
            // sums of the stored (bf16-rounded) values, two columns per op
            const f2v c[2] = {unpack2(o[h][0]), unpack2(o[h][1])};
            if constexpr (EPI == NT_EPI_BIAS_STATS) {
#pragma unroll
              for (int d = 0; d < 2; ++d) {
                const f2v dd = c[d] - bb[d];
                st[0][j][d] += dd;
                st[1][j][d] += dd * dd;
              }
            } else {
              const float4 nm = *reinterpret_cast<const float4*>(nmi_s + j * 16 + q * 4);
              const float4 is = *reinterpret_cast<const float4*>(istd_s + j * 16 + q * 4);
              const f2v nmv[2] = {f2v{nm.x, nm.y}, f2v{nm.z, nm.w}};
              const f2v isv[2] = {f2v{is.x, is.y}, f2v{is.z, is.w}};
#pragma unroll
              for (int d = 0; d < 2; ++d) {
                const f2v xh = unpack2(tf[h][d]) * isv[d] + nmv[d];
                st[0][j][d] += c[d];
                st[1][j][d] += c[d] * xh;
              }
            }
          }
        }
        if constexpr (EPI == NT_EPI_F32) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int n = n0 + (2 * jp + h) * 16 + q * 4;
            __builtin_amdgcn_raw_buffer_store_b128(
                of[h], cr, (mok && n < a.N) ? (int)((m * a.ldc + n) * 4) : OOR, 0, 0);
          }
        } else {
          // rows (q) 0..3 of o[0]/o[1]: after the swap lane row q holds
          // fragment j = 2jp + (q&1), columns 8*(q>>1) .. +7
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            auto sw = __builtin_amdgcn_permlane16_swap(o[0][d], o[1][d], false, false);
            o[0][d] = sw[0];
            o[1][d] = sw[1];
          }
          const u32x4 stv = {o[0][0], o[0][1], o[1][0], o[1][1]};
          const int n = n0 + (2 * jp + (q & 1)) * 16 + (q >> 1) * 8;
          const int64_t ms = (NT_LAB_MODE & 8) ? (m & 4095) : m;   // lab: C writes to a window
          const int off = (mok && n < a.N) ? (int)((ms * a.ldc + n) * 2) : OOR;
          if constexpr (!(NT_LAB_MODE & 1))
            __builtin_amdgcn_raw_buffer_store_b128(stv, cr, off, 0, NT_STORE_AUX);
          else if (acc[i][0][0] == 12345.f)
            __builtin_amdgcn_raw_buffer_store_b128(stv, cr, off, 0, NT_STORE_AUX);
        }
      }
    }
    if constexpr (STATS && !PERSIST) stats_reduce(st, tot, lane);
  }
  if constexpr (STATS) {
    if constexpr (PERSIST) stats_reduce(st, tot, lane);
    // lane (q, m) holds k = bit2(m), j = bit1(m) + 2 bit0(m) + 4 bit3(m),
    // columns 16j + 4q + u.  Sum the waves in fixed order and write this
    // workgroup's partial row part[group][k][n0 + col].
    __syncthreads();   // every wave is done with the W slice: reuse its LDS
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int u = 0; u < 4; ++u) red[(wave * 64 + lane) * 4 + u] = tot[u];
    __syncthreads();
    for (int t = tid; t < 2 * TN; t += NT) {
      const int k = t / TN, col = t % TN;
      const int j = col >> 4, qq = (col >> 2) & 3, u = col & 3;
      const int mm = (k << 2) | (((j >> 2) & 1) << 3) | ((j >> 1) & 1) | ((j & 1) << 1);
      const int ln = qq * 16 + mm;
      float sum = 0.f;
      for (int w = 0; w < NWAVE; ++w) sum += red[(w * 64 + ln) * 4 + u];
      const int n = n0 + col;
      if (n < a.N) a.part[((int64_t)group * 2 + k) * a.N + n] = sum;
    }
  }
}

template <int KTP, int EPI>
dcnr_status launch_nt(NtArgs a, hipStream_t s, int* nparts) {
  using C = NtCfg<KTP>;
  constexpr int NT = Geo<EPI>::NT, TM = Geo<EPI>::TM;
  static bool attr_set = false;
  if (!attr_set) {
    DCNR_HIP(hipFuncSetAttribute((const void*)gemm_nt_kernel<KTP, EPI>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::LDS_BYTES));
    attr_set = true;
  }
  a.nslices = (int)cdiv(a.N, TN);
  // 32-bit buffer offsets: launch in M-chunks of < 2^29 bytes per operand
  const int64_t maxld = std::max<int64_t>({a.ldx, a.ldc * 2, a.R ? a.ldr : 0, a.H ? a.ldh : 0,
                                           a.T ? a.ldt : 0});
  const int64_t mchunk = std::max<int64_t>(TM, ((int64_t(1) << 29) / (maxld * 2)) / TM * TM);
  if (a.M > mchunk) {
    int total = 0;
    for (int64_t m0 = 0; m0 < a.M; m0 += mchunk) {
      NtArgs b = a;
      b.M = std::min(mchunk, a.M - m0);
      b.X = a.X + m0 * a.ldx;
      b.C = (char*)a.C + m0 * a.ldc * (EPI == NT_EPI_F32 ? 4 : 2);
      if (a.R) b.R = (const char*)a.R + m0 * a.ldr * 2;
      if (a.H) b.H = a.H + m0 * a.ldh;
      if (a.T) b.T = a.T + m0 * a.ldt;
      if (a.part) b.part = a.part + (int64_t)total * 2 * a.N;
      int np = 0;
      dcnr_status st = launch_nt<KTP, EPI>(b, s, &np);
      if (st != DCNR_OK) return st;
      total += np;
    }
    if (nparts) *nparts = total;
    return DCNR_OK;
  }
  a.mtiles = cdiv(a.M, TM);
  // one workgroup per CU; grid a multiple of 8 * nslices (XCD grouping)
  const int unit = 8 * a.nslices;
  int grid = std::max(unit, (256 / unit) * unit);
  const int64_t need = a.mtiles * a.nslices;
  if (need < grid) grid = (int)(cdiv(need, unit) * unit);
  a.groups = grid / a.nslices;
  if (nparts) *nparts = a.groups;
  hipLaunchKernelGGL((gemm_nt_kernel<KTP, EPI>), dim3(grid), dim3(NT), C::LDS_BYTES, s, a);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

template <int EPI>
dcnr_status dispatch_k(const NtArgs& a, hipStream_t s, int* nparts) {
  if (a.K <= 128) return launch_nt<4, EPI>(a, s, nparts);
  if (a.K <= 256) return launch_nt<8, EPI>(a, s, nparts);
  return launch_nt<16, EPI>(a, s, nparts);
}

}  // namespace

bool gemm_nt_supported(int64_t K, int64_t N) { return K <= 512 && K % 8 == 0 && N % 8 == 0; }

// Upper bound of the part rows a stats epilogue writes (workspace sizing).
int gemm_nt_max_parts(int64_t M, int N) {
  const int64_t chunks =
      cdiv(M, std::max<int64_t>(TM_MIN, ((int64_t(1) << 29) / (1024 * 2)) / TM_MIN * TM_MIN)) + 1;
  return (int)(chunks * std::max<int64_t>(256 / (8 * cdiv(N, TN)), 1) * 8);
}

dcnr_status gemm_nt(int epi, const NtArgs& a, hipStream_t s, int* nparts) {
  if (nparts) *nparts = 0;
  if (a.fin) {
    set_error("gemm_nt: no in-kernel finalize (use gemm_ws)");
    return DCNR_BAD_ARG;
  }
  if (a.M <= 0 || a.N <= 0) return DCNR_OK;
  const bool ht = epi == NT_EPI_RESID_BN || epi == NT_EPI_DROP_BN;
  if (!gemm_nt_supported(a.K, a.N) || a.ldx % 8 || a.ldw % 8 || a.ldc % 8 ||
      ((epi == NT_EPI_RESID || epi == NT_EPI_RESID_BN) && (a.ldr % 8 || !a.R)) ||
      (ht && (!a.H || !a.T || !a.mean || !a.invstd || a.ldh % 4 || a.ldt % 4)) ||
      (nt_epi_stats(epi) && !a.part)) {
    set_error("gemm_nt: unsupported K=%d N=%d / missing epilogue operand", a.K, a.N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  switch (epi) {
    case NT_EPI_BIAS: return dispatch_k<NT_EPI_BIAS>(a, s, nparts);
    case NT_EPI_F32: return dispatch_k<NT_EPI_F32>(a, s, nparts);
    case NT_EPI_RESID: return dispatch_k<NT_EPI_RESID>(a, s, nparts);
    case NT_EPI_BIAS_STATS: return dispatch_k<NT_EPI_BIAS_STATS>(a, s, nparts);
    case NT_EPI_RESID_BN: return dispatch_k<NT_EPI_RESID_BN>(a, s, nparts);
    case NT_EPI_DROP_BN: return dispatch_k<NT_EPI_DROP_BN>(a, s, nparts);
  }
  set_error("gemm_nt: bad epilogue");
  return DCNR_BAD_ARG;
}

}  // namespace dcnr
