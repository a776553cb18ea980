// Weight-stationary streaming GEMM for the bf16 deep tower (gfx950):
//
//   C[M, N] = X[M, K] . W[N, K]^T  (+ epilogue),  K <= 512
//
// The deep tower's Linear layers (train.py:143,105,109) have a huge M (the
// batch) and a small N x K weight: one pass over the activations.  Compared
// with gemm_nt.hip (W slice in LDS, X fragments streamed per wave) this
// kernel halves the X bytes each CU has to pull per FLOP (measured in round 1;
// the W-in-LDS kernel has been retired):
//  * a workgroup owns a 256-column slice of W and keeps it in REGISTERS for
//    its whole lifetime: each of the 8 waves holds 32 columns x K as MFMA
//    A-operand fragments (K = 512: 128 VGPRs per lane);
//  * the X tile (64 rows x K) is staged once per workgroup into LDS by
//    LDS-DMA (buffer_load ... lds, double-buffered, one barrier per tile) and
//    read by all 8 waves as MFMA B-operand fragments (ds_read_b128, chunk
//    XOR-swizzled by row: conflict-free);
//  * so X is read from L2 twice for N = 512 (two slices, on one XCD), not
//    four times, and the per-CU vector-memory traffic per FLOP halves;
//  * v_mfma_f32_16x16x32_bf16 with W as A: each lane accumulates 4
//    consecutive output columns of one row; the epilogue pairs the wave's two
//    16-column blocks with v_permlane16_swap into 16-byte row-contiguous
//    stores (and loads its operands the same way);
//  * the BatchNorm-statistics epilogues keep per-lane column partials in
//    registers over all of the workgroup's tiles (each wave owns its columns:
//    no cross-wave reduction) and write one partial row per workgroup;
//  * eval: BN (from the running statistics, computed per column at launch)
//    + ReLU (+ residual) in the epilogue, and for the last residual block the
//    deep head dot (NT_EPI_BN_RESID_RELU_HEAD: one partial per row and wave,
//    no C store).
#include "dcnr_internal.h"

#include <type_traits>

namespace dcnr {
namespace {

// Per-epilogue tile rows and operand-load placement (measured with
// tools/ws_lab.hip in rounds 2-3, removed since in commit 77025d0, M = 131072, K = N = 512): 64-row tiles where
// registers allow; the epilogues with operands use 32-row tiles and issue
// every operand load before the MFMAs ("early": RESID 90.5 vs 96.4 us one row
// block ahead, DROP_BN 104.7 vs 111.9 us at 64 rows); eval BN_RELU at 32 rows
// (71.5 vs 75.4-77.2 us at 64).  Rejected variants (stagger, software-pipelined
// epilogue, two 4-wave workgroups per CU, static priority, deeper fragment
// prefetch, in-launch BN reduction) and their numbers: DESIGN.md section 8.
constexpr int WS_WAVES = 8, WS_NT = 64 * WS_WAVES, WS_WC = 32, WS_TN = WS_WAVES * WS_WC;
constexpr int WS_PFD = 1;   // fragment prefetch distance of the MFMA loop, in K steps
template <int KTP, int EPI> constexpr int ws_tm() {
  return EPI <= NT_EPI_F32 || EPI == NT_EPI_BIAS_STATS ? 64 : 32;
}
template <int EPI> constexpr bool ws_ops_early() {
  return EPI == NT_EPI_RESID || EPI == NT_EPI_RESID_BN || EPI == NT_EPI_DROP_BN || EPI == NT_EPI_BN_RESID_RELU ||
         EPI == NT_EPI_BN_RESID_RELU_HEAD || EPI == NT_EPI_RESID_SUM;
}
// X-tile buffers in the LDS ring: one tile in flight while one is consumed.
constexpr int WS_NB = 2;

template <int KTP, int TM, int NB = WS_NB> struct WsCfg {
  static constexpr int P = KTP * 64;                      // LDS bytes per X row
  static constexpr int CPR = KTP * 4;                     // 16-B chunks per row
  static constexpr int TILE = TM * P;                     // bytes per X buffer
  static constexpr int RPD = 1024 / P;                    // rows per DMA wave-instruction
  static constexpr int DPW = TM / RPD / WS_WAVES;         // DMAs per wave per tile
  static constexpr int RB = TM / 16;                      // 16-row blocks per tile
  static constexpr size_t LDS_BYTES = NB * (size_t)TILE + 4 * WS_TN * 4;
  static_assert(TM % (RPD * WS_WAVES) == 0 && TM % 16 == 0, "tile rows");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

typedef float f2v __attribute__((ext_vector_type(2)));

typedef bf16 bf16x2v __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 (round to nearest even) in ONE v_cvt_pk_bf16_f32
// (the scalar casts cost two conversions + a shift + an or)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{a, b}, bf16x2v));
}
__device__ __forceinline__ f2v unpack2(uint32_t w) {
  return f2v{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
// store layout (16 B per lane: columns 16(q&1) + 8(q>>1) .. +7 of the wave's
// 32) <-> accumulator layout of the two column blocks (columns 16cb + 4q ..)
__device__ __forceinline__ void to_acc_layout(const u32x4& L, u32x2 (&f)[2]) {
  auto a = __builtin_amdgcn_permlane16_swap(L[0], L[2], false, false);
  auto b = __builtin_amdgcn_permlane16_swap(L[1], L[3], false, false);
  f[0] = u32x2{a[0], b[0]};
  f[1] = u32x2{a[1], b[1]};
}
template <int H, int CTRL>
__device__ __forceinline__ void bfly(float (&x)[16], bool hi) {
#pragma unroll
  for (int u = 0; u < H; ++u) {
    const float give = hi ? x[u] : x[u + H];
    const float keep = hi ? x[u + H] : x[u];
    x[u] = keep + dpp<CTRL>(give);
  }
}

// X tile rows m0 .. m0+63 -> LDS buffer `dst` (row r at r*P, 16-B chunk c at
// position c ^ (r & 15)); xr covers rows from m0 on (rows >= M read 0).
// (Lane offsets recomputed per tile: registers are the scarce resource here.)
template <int KTP, int TM>
__device__ __forceinline__ void issue_tile(u32x4 xr, int64_t ldx, int K, uint32_t dst, int wave,
                                           int lane) {
  using C = WsCfg<KTP, TM>;
#pragma unroll
  for (int d = 0; d < C::DPW; ++d) {
    const int r = (wave * C::DPW + d) * C::RPD + lane / C::CPR;
    const int c = (lane % C::CPR) ^ (r & 15);
    const int off = c * 8 < K ? (int)(((int64_t)r * ldx + c * 8) * 2) : OOR;
    dma16(xr, off, dst + (wave * C::DPW + d) * 1024);
  }
}

// XBN (RESID_BN / DROP_BN at K = 512): the operand transform of NtArgs.Tx --
// each X tile's du and t are DMA'd side by side, the workgroup turns du into
// dt in LDS (bn_bwd_dt, per-column constants in LDS) before the MFMAs read
// it, and slice 0's workgroups store dt for the weight gradient.  This takes
// the BatchNorm backward's row pass (read du and t, write dt) and the GEMM's
// re-read of dt off the backward: one kernel reads du and t once.
template <int KTP, int EPI, bool XBN = false>
__global__ __launch_bounds__(WS_NT, 1) void gemm_ws_kernel(NtArgs a) {
  constexpr int WS_TM = ws_tm<KTP, EPI>();
  constexpr int NB = WS_NB;
  using C = WsCfg<KTP, WS_TM, NB>;
  constexpr int WS_RB = C::RB;
  constexpr bool STATS = (EPI >= NT_EPI_BIAS_STATS && EPI <= NT_EPI_DROP_BN) || EPI == NT_EPI_RESID_SUM;
  constexpr bool HEAD = EPI == NT_EPI_BN_RESID_RELU_HEAD;
  constexpr bool HAS_R = EPI == NT_EPI_RESID || EPI == NT_EPI_RESID_BN || EPI == NT_EPI_BN_RESID_RELU || HEAD ||
                         EPI == NT_EPI_RESID_SUM;
  constexpr bool HAS_HT = EPI == NT_EPI_RESID_BN || EPI == NT_EPI_DROP_BN;
  constexpr bool HAS_SS = EPI >= NT_EPI_BN_RELU && EPI <= NT_EPI_BN_RESID_RELU_HEAD;   // eval BN affine + ReLU
  constexpr bool HAS_BIAS = EPI <= NT_EPI_BIAS_STATS || HAS_SS;
  static_assert(!XBN || (WS_NT % C::CPR == 0 && (HAS_HT || EPI == NT_EPI_RESID || EPI == NT_EPI_RESID_SUM)),
                "operand transform: dX epilogues, whole rows");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, l15 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nsl = a.nslices, bid = blockIdx.x;
  const int slice = (bid / 8) % nsl;
  const int group = (bid % 8) + 8 * (bid / (8 * nsl));
  const int groups = a.groups;
  const int n0 = slice * WS_TN;
  const int nw = n0 + wave * WS_WC;   // this wave's first column

  // first tile's DMA goes out before anything else
  auto tile_rsrc = [&](int64_t mt) {
    const int64_t m0 = mt * WS_TM;
    const int64_t rows = a.M - m0;
    return rsrc_words(a.X + m0 * a.ldx, rows > 0 ? rows * a.ldx * 2 : 0);
  };
  const uint32_t lbase = lds_addr(lds);
  // XBN: the t tiles after the X tiles and the slice constants
  constexpr int XOFF = NB * C::TILE + 4 * WS_TN * 4;
  auto ttile_rsrc = [&](int64_t mt) {
    const int64_t m0 = mt * WS_TM;
    const int64_t rows = a.M - m0;
    return rsrc_words(a.Tx + m0 * a.ldx, rows > 0 ? rows * a.ldx * 2 : 0);
  };
#pragma unroll
  for (int j = 0; j < NB - 1; ++j)
    if (group + (int64_t)j * groups < a.mtiles) {
      issue_tile<KTP, WS_TM>(tile_rsrc(group + (int64_t)j * groups), a.ldx, a.K, lbase + j * C::TILE,
                             wave, lane);
      if constexpr (XBN)
        issue_tile<KTP, WS_TM>(ttile_rsrc(group + (int64_t)j * groups), a.ldx, a.K,
                               lbase + XOFF + j * C::TILE, wave, lane);
    }

  // resident W: fragments (column block cb, k-step kt) of columns nw + 16cb + l15
  bf16x8 wf[2][KTP];
  {
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.W, (short)0, (int)((int64_t)a.N * a.ldw * 2), 0x00020000);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int n = nw + cb * 16 + l15;
#pragma unroll
      for (int kt = 0; kt < KTP; ++kt) {
        const int k = kt * 32 + 8 * q;
        const bool ok = n < a.N && k < a.K;
        wf[cb][kt] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, ok ? (int)(((int64_t)n * a.ldw + k) * 2) : OOR, 0, 0));
      }
    }
  }
  // per-column constants of the slice: bias, -mean*invstd, invstd (eval BN:
  // scale, shift)
  float* bias_s = reinterpret_cast<float*>(lds + NB * C::TILE);
  float* nmi_s = bias_s + WS_TN;
  float* istd_s = bias_s + 2 * WS_TN;
  float* wf_s = bias_s + 3 * WS_TN;   // HEAD: the slice's deep head weights
  for (int c = tid; c < WS_TN; c += WS_NT) {
    const int n = n0 + c;
    bias_s[c] = (HAS_BIAS && a.bias && n < a.N) ? a.bias[n] : 0.f;
    if constexpr (HAS_HT) {
      nmi_s[c] = n < a.N ? -a.mean[n] * a.invstd[n] : 0.f;
      istd_s[c] = n < a.N ? a.invstd[n] : 0.f;
    }
    if constexpr (HAS_SS) {
      if (a.bn_rm) {   // running-stat affine, as bn_eval_multi_kernel (pads: 0)
        float sc = 0.f, sh = 0.f;
        if (n < a.Nr) {
          const double mean = a.bn_rm[n], var = a.bn_rv[n];
          const float inv = (float)(1.0 / sqrt(var + (double)BN_EPS));
          sc = a.bn_g[n] * inv;
          sh = a.bn_b[n] - (float)mean * sc;
        }
        nmi_s[c] = sc;
        istd_s[c] = sh;
      } else {
        nmi_s[c] = n < a.N ? a.bn_scale[n] : 0.f;
        istd_s[c] = n < a.N ? a.bn_shift[n] : 0.f;
      }
    }
    if constexpr (HEAD) wf_s[c] = n < a.Nr ? a.wf[n] : 0.f;
  }
  // XBN: the transform's per-column constants [mean, invstd, k0, k1, k2][K]
  float* xc_s = reinterpret_cast<float*>(lds + XOFF + NB * C::TILE);
  if constexpr (XBN) {
    for (int c = tid; c < KTP * 32; c += WS_NT) {
      const bool ok = c < a.K;
      xc_s[c] = ok ? a.xmean[c] : 0.f;
      xc_s[KTP * 32 + c] = ok ? a.xinvstd[c] : 0.f;
      xc_s[2 * KTP * 32 + c] = ok ? a.xcoef[c] : 0.f;
      xc_s[3 * KTP * 32 + c] = ok ? a.xcoef[a.K + c] : 0.f;
      xc_s[4 * KTP * 32 + c] = ok ? a.xcoef[2 * a.K + c] : 0.f;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int es = EPI == NT_EPI_F32 ? 4 : 2;
  const __amdgpu_buffer_rsrc_t cr =
      __builtin_amdgcn_make_buffer_rsrc(a.C, (short)0, (int)(a.M * a.ldc * es), 0x00020000);
  const __amdgpu_buffer_rsrc_t rr_ = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.R, (short)0, HAS_R ? (int)(a.M * a.ldr * 2) : 0, 0x00020000);
  // 1-bit keep mask (a.Hb): bit c%32 of word [m][c/32]
  const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.Hb, (short)0, HAS_HT ? (int)(a.M * a.ldhb * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.T, (short)0, HAS_HT ? (int)(a.M * a.ldt * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t hp_r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.headp, (short)0, HEAD ? (int)(((a.nslices * WS_WAVES - 1) * a.ldh + a.M) * 4) : 0, 0x00020000);

  // per-lane column partials [sum, sum2][cb][column pair], over all tiles
  f2v st[2][2][2];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 2; ++r) st[k][cb][r] = f2v{0.f, 0.f};

  // fragment read offsets: row rb*16 + l15, chunk (4kt + q) ^ l15
  const uint32_t rowoff = (uint32_t)l15 * C::P;
  int coff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) coff[j] = ((4 * j + q) ^ l15) * 16;
  const int nst = nw + (q & 1) * 16 + (q >> 1) * 8;   // store-layout column
  // epilogue operands (WS_OPS_EARLY: all issued before the MFMAs, else one
  // row block ahead of their use)
  constexpr bool WS_OPS_EARLY = ws_ops_early<EPI>();
  constexpr int NSLOT = WS_OPS_EARLY ? WS_RB : 2;
  u32x4 rv[NSLOT], tv[NSLOT];
  uint32_t hw[NSLOT];   // the mask word of columns nw .. nw+31
  auto load_ops = [&](int64_t m0, int rb, int slot) {
    const int64_t m = m0 + rb * 16 + l15;
    const bool ok = m < a.M && nst < a.N;
    if constexpr (HAS_R)
      rv[slot] = __builtin_amdgcn_raw_buffer_load_b128(rr_, ok ? (int)((m * a.ldr + nst) * 2) : OOR, 0, 0);
    if constexpr (HAS_HT) {
      hw[slot] = __builtin_amdgcn_raw_buffer_load_b32(
          hr, (m < a.M && nw < a.N) ? (int)((m * a.ldhb + (nw >> 5)) * 4) : OOR, 0, 0);
      tv[slot] = __builtin_amdgcn_raw_buffer_load_b128(tr, ok ? (int)((m * a.ldt + nst) * 2) : OOR, 0, 0);
    }
  };
  f32x4 acc[WS_RB][2];
  // ---- epilogue of row block rb of the tile at row m0 (accumulators ac, its
  // operands in the slots)
  auto epi_rb = [&](const int64_t m0, const int rb, f32x4 (&ac)[WS_RB][2]) {
    // lane holds C[m][nw + 16cb + 4q .. +3], m = m0 + 16rb + l15
    {
      const int64_t m = m0 + rb * 16 + l15;
      const bool mok = m < a.M;
      if (!WS_OPS_EARLY && rb + 1 < WS_RB) load_ops(m0, rb + 1, (rb + 1) & 1);
      const int slot = WS_OPS_EARLY ? rb : rb & 1;
      u32x2 o[2], rf[2], tf[2];
      u32x4 of[2];
      float hd = 0.f;   // HEAD: this lane's 8 columns of the row's dot
      if constexpr (HAS_R) to_acc_layout(rv[slot], rf);
      if constexpr (HAS_HT) to_acc_layout(tv[slot], tf);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int cl = wave * WS_WC + cb * 16 + q * 4;   // column within the slice
        f2v v[2] = {f2v{ac[rb][cb][0], ac[rb][cb][1]}, f2v{ac[rb][cb][2], ac[rb][cb][3]}};
        f2v bb[2];
        if constexpr (HAS_BIAS) {
          const float4 bj = *reinterpret_cast<const float4*>(bias_s + cl);
          bb[0] = f2v{bj.x, bj.y};
          bb[1] = f2v{bj.z, bj.w};
          v[0] += bb[0];
          v[1] += bb[1];
        }
        if constexpr (HAS_SS) {
          const float4 sc = *reinterpret_cast<const float4*>(nmi_s + cl);
          const float4 sh = *reinterpret_cast<const float4*>(istd_s + cl);
          v[0] = v[0] * f2v{sc.x, sc.y} + f2v{sh.x, sh.y};
          v[1] = v[1] * f2v{sc.z, sc.w} + f2v{sh.z, sh.w};
        }
        if constexpr (HAS_R) {
#pragma unroll
          for (int d = 0; d < 2; ++d) v[d] += unpack2(rf[cb][d]);
        }
        if constexpr (HAS_SS) {
#pragma unroll
          for (int d = 0; d < 2; ++d) v[d] = f2v{relu_f(v[d][0]), relu_f(v[d][1])};
        }
        if constexpr (EPI == NT_EPI_DROP_BN) {
          v[0] *= a.hscale;
          v[1] *= a.hscale;
        }
        o[cb] = u32x2{pack2(v[0][0], v[0][1]), pack2(v[1][0], v[1][1])};
        if constexpr (HEAD) {   // the stored (bf16-rounded) activation, as row_dot reads it
          const float4 w4 = *reinterpret_cast<const float4*>(wf_s + cl);
          const f2v c0 = unpack2(o[cb][0]), c1 = unpack2(o[cb][1]);
          hd += ((c0[0] * w4.x + c0[1] * w4.y) + c1[0] * w4.z) + c1[1] * w4.w;
        }
        of[cb] = u32x4{__float_as_uint(v[0][0]), __float_as_uint(v[0][1]),
                       __float_as_uint(v[1][0]), __float_as_uint(v[1][1])};
        if constexpr (HAS_HT) {
          // RESID_BN: keep where h > 0 (bf16 bits: magnitude != 0, sign clear);
          // DROP_BN: keep where h != 0 (the saved dropout activation)
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            // bits 16cb + 4q + 2d (+1) of the wave's 32 columns
            const uint32_t kb = hw[slot] >> (16 * cb + 4 * q + 2 * d);
            o[cb][d] &= ((kb & 1u) * 0xffffu) | (((kb >> 1) & 1u) * 0xffff0000u);
          }
        }
        if constexpr (STATS) {
          // sums of the stored (bf16-rounded) values
          if (mok) {
            const f2v c[2] = {unpack2(o[cb][0]), unpack2(o[cb][1])};
            if constexpr (EPI == NT_EPI_BIAS_STATS || EPI == NT_EPI_RESID_SUM) {
#pragma unroll
              for (int d = 0; d < 2; ++d) {
                f2v dd = c[d];
                if constexpr (HAS_BIAS) dd -= bb[d];
                st[0][cb][d] += dd;
                st[1][cb][d] += dd * dd;
              }
            } else {
              const float4 nm = *reinterpret_cast<const float4*>(nmi_s + cl);
              const float4 is = *reinterpret_cast<const float4*>(istd_s + cl);
              const f2v nmv[2] = {f2v{nm.x, nm.y}, f2v{nm.z, nm.w}};
              const f2v isv[2] = {f2v{is.x, is.y}, f2v{is.z, is.w}};
#pragma unroll
              for (int d = 0; d < 2; ++d) {
                const f2v xh = unpack2(tf[cb][d]) * isv[d] + nmv[d];
                st[0][cb][d] += c[d];
                st[1][cb][d] += c[d] * xh;
              }
            }
          }
        }
      }
      if constexpr (HEAD) {
        // the row's 4 lanes (q = 0..3, same l15): half-wave then row swap
        const unsigned u = __float_as_uint(hd);
        auto h2 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        const float t = __uint_as_float(h2[0]) + __uint_as_float(h2[1]);
        const unsigned ut = __float_as_uint(t);
        auto h4 = __builtin_amdgcn_permlane16_swap(ut, ut, false, false);
        const float r4 = __uint_as_float(h4[0]) + __uint_as_float(h4[1]);
        if (q == 0)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r4), hp_r,
                                                mok ? (int)(((slice * WS_WAVES + wave) * a.ldh + m) * 4) : OOR, 0, 0);
      } else if constexpr (EPI == NT_EPI_F32) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const int n = nw + cb * 16 + q * 4;
          __builtin_amdgcn_raw_buffer_store_b128(
              of[cb], cr, (mok && n < a.N) ? (int)((m * a.ldc + n) * 4) : OOR, 0, 0);
        }
      } else {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          auto sw = __builtin_amdgcn_permlane16_swap(o[0][d], o[1][d], false, false);
          o[0][d] = sw[0];
          o[1][d] = sw[1];
        }
        const u32x4 sv = {o[0][0], o[0][1], o[1][0], o[1][1]};
        const int off = (mok && nst < a.N) ? (int)((m * a.ldc + nst) * 2) : OOR;
        __builtin_amdgcn_raw_buffer_store_b128(sv, cr, off, 0, 0);
      }
    }
  };
  // ---- epilogue of the whole tile at row m0
  auto epilogue = [&](const int64_t m0, f32x4 (&ac)[WS_RB][2]) {
#pragma unroll
    for (int rb = 0; rb < WS_RB; ++rb) epi_rb(m0, rb, ac);
  };

  int buf = 0;
  for (int64_t mt = group; mt < a.mtiles; mt += groups, buf = buf + 1 == NB ? 0 : buf + 1) {
    const int64_t mn = mt + (int64_t)(NB - 1) * groups;
    const int nbuf = buf + NB - 1 >= NB ? buf - 1 : buf + NB - 1;   // (buf + NB - 1) % NB
    if (mn < a.mtiles) {
      issue_tile<KTP, WS_TM>(tile_rsrc(mn), a.ldx, a.K, lbase + nbuf * C::TILE, wave, lane);
      if constexpr (XBN)
        issue_tile<KTP, WS_TM>(ttile_rsrc(mn), a.ldx, a.K, lbase + XOFF + nbuf * C::TILE, wave, lane);
    }
    const int64_t m0 = mt * WS_TM;
    if constexpr (XBN) {
      // du -> dt in place in this tile's LDS image (16-B chunk c of row r at
      // position c ^ (r & 15)); a thread keeps one column group (WS_NT is a
      // multiple of the chunks per row), so its constants are read once
      char* xt = lds + buf * C::TILE;
      const char* tt = lds + XOFF + buf * C::TILE;
      const int cg = tid % C::CPR;
      float mu[8], is[8], k0[8], k1[8], k2[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        mu[v] = xc_s[cg * 8 + v];
        is[v] = xc_s[KTP * 32 + cg * 8 + v];
        k0[v] = xc_s[2 * KTP * 32 + cg * 8 + v];
        k1[v] = xc_s[3 * KTP * 32 + cg * 8 + v];
        k2[v] = xc_s[4 * KTP * 32 + cg * 8 + v];
      }
      const __amdgpu_buffer_rsrc_t dr = buf_rsrc(a.dt + m0 * a.ldx, slice == 0 ? (a.M - m0) * a.ldx * 2 : 0);
#pragma unroll
      for (int e = tid; e < WS_TM * C::CPR; e += WS_NT) {
        const int r = e / C::CPR;
        const int pos = r * C::P + ((cg ^ (r & 15)) << 4);
        const u32x4 u = *reinterpret_cast<const u32x4*>(xt + pos);
        const u32x4 t = *reinterpret_cast<const u32x4*>(tt + pos);
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f2v uu = unpack2(u[j]), tv2 = unpack2(t[j]);
          o[j] = pack2(bn_bwd_dt(uu[0], tv2[0], mu[2 * j], is[2 * j], k0[2 * j], k1[2 * j], k2[2 * j]),
                       bn_bwd_dt(uu[1], tv2[1], mu[2 * j + 1], is[2 * j + 1], k0[2 * j + 1], k1[2 * j + 1],
                                 k2[2 * j + 1]));
        }
        *reinterpret_cast<u32x4*>(xt + pos) = o;
        // (rows past M: 0 bytes of descriptor, the store is dropped; chunks
        // past K are not columns of the row: K < 512 would write them into
        // the next row)
        __builtin_amdgcn_raw_buffer_store_b128(o, dr, cg * 8 < a.K ? (int)((r * a.ldx + cg * 8) * 2) : OOR, 0,
                                               0);
      }
      __syncthreads();
    }
    if constexpr (WS_OPS_EARLY) {
#pragma unroll
      for (int rb = 0; rb < WS_RB; ++rb) load_ops(m0, rb, rb);
    } else {
      load_ops(m0, 0, 0);
    }
    const char* xb = lds + buf * C::TILE + rowoff;
#pragma unroll
    for (int rb = 0; rb < WS_RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fragment (kt, rb): row rb*16 + l15, physical chunk (4kt + q) ^ l15 =
    // 16 (kt >> 2) + coff[kt & 3]: 4 offset registers, the rest immediates
    auto xrd = [&](int kt, int rb) {
      return *reinterpret_cast<const bf16x8*>(xb + rb * 16 * C::P + (kt >> 2) * 256 + coff[kt & 3]);
    };
    // fragments of step kt sit in buffer kt % NXB, read WS_PFD steps ahead
    constexpr int NXB = WS_PFD + 1;
    bf16x8 xf[NXB][WS_RB];
#pragma unroll
    for (int p = 0; p < WS_PFD; ++p)
#pragma unroll
      for (int rb = 0; rb < WS_RB; ++rb) xf[p][rb] = xrd(p, rb);
#pragma unroll
    for (int kt = 0; kt < KTP; ++kt) {
      const int cur = kt % NXB;
      const bool rd = kt + WS_PFD < KTP;
      if (rd) {
#pragma unroll
        for (int rb = 0; rb < WS_RB; ++rb) xf[(kt + WS_PFD) % NXB][rb] = xrd(kt + WS_PFD, rb);
      }
#pragma unroll
      for (int rb = 0; rb < WS_RB; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][kt], xf[cur][rb], acc[rb][cb], 0, 0, 0);
      // keep step kt+PFD's fragment reads in step kt (PFD full steps of MFMAs
      // between a read and its use), spread between the MFMAs
      if (rd) {
#pragma unroll
        for (int rb = 0; rb < WS_RB; ++rb) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMA
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    epilogue(m0, acc);
    // next tile's X landed and every wave is done reading this buffer.  Younger
    // than the next tile's DMAs: the stores of the last NB-1 tiles and the
    // DMAs of the NB-2 tiles after it -- when all of those were issued (near
    // the end some prefetches are not) the count below is exact, else wait all
    constexpr int NSTORE = (EPI == NT_EPI_F32 ? 2 : 1) * WS_RB;
    constexpr int NWAIT = (NB - 1) * NSTORE + (NB - 2) * C::DPW;
    if (NB == 2 || mn < a.mtiles)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NWAIT) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if constexpr (STATS) {
    // 16-lane butterfly: lane (q, m) ends with k = bit2(m), cb = bit3(m),
    // column pair element r = 2 bit0(m) + bit1(m) of columns nw + 16cb + 4q
    float x[16];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[k * 8 + cb * 4 + r] = st[k][cb][r >> 1][r & 1];
    bfly<8, 0x141>(x, (lane & 4) != 0);   // partner lane^7, keep by bit 2
    bfly<4, 0x128>(x, (lane & 8) != 0);   // lane^8, bit 3
    bfly<2, 0xB1>(x, (lane & 1) != 0);    // lane^1, bit 0
    bfly<1, 0x4E>(x, (lane & 2) != 0);    // lane^2, bit 1
    const int k = (lane >> 2) & 1, cb = (lane >> 3) & 1, r = 2 * (lane & 1) + ((lane >> 1) & 1);
    const int n = nw + cb * 16 + q * 4 + r;
    if (n < a.N) a.part[((int64_t)group * 2 + k) * a.N + n] = x[0];
  }
}

template <int KTP, int EPI, bool XBN = false>
dcnr_status launch_ws(NtArgs a, hipStream_t s, int* nparts) {
  constexpr int WS_TM = ws_tm<KTP, EPI>();
  using C = WsCfg<KTP, WS_TM>;
  // XBN: + the t tiles and the transform's 5 x K constants
  constexpr size_t LDSB = C::LDS_BYTES + (XBN ? WS_NB * (size_t)C::TILE + 5 * KTP * 32 * 4 : 0);
  static_assert(LDSB <= 160 * 1024, "LDS budget");
  TRY_ST(set_max_dyn_lds((const void*)gemm_ws_kernel<KTP, EPI, XBN>, LDSB));
  a.nslices = (int)cdiv(a.N, WS_TN);
  // 32-bit buffer offsets: launch in M-chunks of < 2^29 bytes per operand
  const int64_t maxld = std::max<int64_t>({a.ldx, a.ldc * 2, a.R ? a.ldr : 0, a.Hb ? a.ldhb * 2 : 0,
                                           a.T ? a.ldt : 0});
  const int64_t mchunk = std::max<int64_t>(WS_TM, ((int64_t(1) << 29) / (maxld * 2)) / WS_TM * WS_TM);
  if (a.M > mchunk) {
    int total = 0;
    for (int64_t m0 = 0; m0 < a.M; m0 += mchunk) {
      NtArgs b = a;
      b.M = std::min(mchunk, a.M - m0);
      b.X = a.X + m0 * a.ldx;
      b.C = (char*)a.C + m0 * a.ldc * (EPI == NT_EPI_F32 ? 4 : 2);
      if (a.R) b.R = (const char*)a.R + m0 * a.ldr * 2;
      if (a.Hb) b.Hb = a.Hb + m0 * a.ldhb;
      if (a.headp) b.headp = a.headp + m0;   // same row stride ldh
      if (a.T) b.T = a.T + m0 * a.ldt;
      if (a.Tx) b.Tx = a.Tx + m0 * a.ldx;
      if (a.dt) b.dt = a.dt + m0 * a.ldx;
      if (a.part) b.part = a.part + (int64_t)total * 2 * a.N;
      int np = 0;
      dcnr_status st = launch_ws<KTP, EPI, XBN>(b, s, &np);
      if (st != DCNR_OK) return st;
      total += np;
    }
    if (nparts) *nparts = total;
    return DCNR_OK;
  }
  a.mtiles = cdiv(a.M, WS_TM);
  const int unit = 8 * a.nslices;
  // (XBN: the workgroups could leave XBN_FREE CUs to the side stream's
  // weight gradients, which cannot share a CU with this kernel's registers
  // and LDS: 32 / 64 / 96 / 128 measured level / level / level / +5 % per
  // step, profiles/lab/r06_xbn_lab.txt)
  constexpr int XBN_FREE = 0;
  int grid = std::max(unit, ((256 - (XBN ? XBN_FREE : 0)) / unit) * unit);
  const int64_t need = a.mtiles * a.nslices;
  if (need < grid) grid = (int)(cdiv(need, unit) * unit);
  a.groups = grid / a.nslices;
  if (nparts) *nparts = a.groups;
  hipLaunchKernelGGL((gemm_ws_kernel<KTP, EPI, XBN>), dim3(grid), dim3(WS_NT), LDSB, s, a);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

template <int EPI>
dcnr_status dispatch_ws(const NtArgs& a, hipStream_t s, int* nparts) {
  if (a.K <= 128) return launch_ws<4, EPI>(a, s, nparts);
  if (a.K <= 256) return launch_ws<8, EPI>(a, s, nparts);
  return launch_ws<16, EPI>(a, s, nparts);
}

}  // namespace

bool gemm_ws_supported(int64_t K, int64_t N) { return K <= 512 && K % 8 == 0 && N % 8 == 0; }
bool gemm_ws_xbn_supported(int epi, int64_t K, int64_t N) {
  return (epi == NT_EPI_RESID_BN || epi == NT_EPI_DROP_BN || epi == NT_EPI_RESID || epi == NT_EPI_RESID_SUM) &&
         K > 256 && K <= 512 &&
         K % 8 == 0 && N % 8 == 0;
}
int gemm_ws_head_parts(int64_t N) { return N % 8 == 0 && N <= 4096 ? (int)cdiv(N, WS_TN) * WS_WAVES : 0; }

dcnr_status gemm_ws(int epi, const NtArgs& a, hipStream_t s, int* nparts) {
  if (nparts) *nparts = 0;
  if (a.M <= 0 || a.N <= 0) return DCNR_OK;
  const bool ht = epi == NT_EPI_RESID_BN || epi == NT_EPI_DROP_BN;
  if (!gemm_ws_supported(a.K, a.N) || a.ldx % 8 || a.ldw % 8 || a.ldc % 8 ||
      ((epi == NT_EPI_RESID || epi == NT_EPI_RESID_BN || epi == NT_EPI_BN_RESID_RELU || epi == NT_EPI_RESID_SUM) &&
       (a.ldr % 8 || !a.R)) ||
      (epi >= NT_EPI_BN_RELU && epi <= NT_EPI_BN_RESID_RELU_HEAD && !a.bn_rm && (!a.bn_scale || !a.bn_shift)) ||
      (epi >= NT_EPI_BN_RELU && epi <= NT_EPI_BN_RESID_RELU_HEAD && a.bn_rm && (!a.bn_g || !a.bn_b || !a.bn_rv)) ||
      (epi == NT_EPI_BN_RESID_RELU_HEAD &&
       (!a.wf || !a.headp || !gemm_ws_head_parts(a.N) || a.ldh < a.M ||
        a.ldh * gemm_ws_head_parts(a.N) * 4 >= (int64_t(1) << 31))) ||
      (ht && (!a.Hb || !a.T || !a.mean || !a.invstd || a.ldt % 8)) ||
      (nt_epi_stats(epi) && !a.part)) {
    set_error("gemm_ws: unsupported K=%d N=%d / missing epilogue operand", a.K, a.N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (a.Tx) {   // the dX GEMMs with the BatchNorm backward's row pass folded in
    if (!gemm_ws_xbn_supported(epi, a.K, a.N) || !a.dt || !a.xmean || !a.xinvstd || !a.xcoef) {
      set_error("gemm_ws: unsupported operand transform (epi %d K=%d N=%d)", epi, a.K, a.N);
      return DCNR_UNSUPPORTED_SHAPE;
    }
    if (epi == NT_EPI_RESID_SUM) return launch_ws<16, NT_EPI_RESID_SUM, true>(a, s, nparts);
    if (epi == NT_EPI_RESID) return launch_ws<16, NT_EPI_RESID, true>(a, s, nparts);
    return epi == NT_EPI_RESID_BN ? launch_ws<16, NT_EPI_RESID_BN, true>(a, s, nparts)
                                  : launch_ws<16, NT_EPI_DROP_BN, true>(a, s, nparts);
  }
  if (gemm_wsp_supported(epi, a.K, a.N)) return gemm_wsp(epi, a, s, nparts);
  switch (epi) {
    case NT_EPI_BIAS: return dispatch_ws<NT_EPI_BIAS>(a, s, nparts);
    case NT_EPI_F32: return dispatch_ws<NT_EPI_F32>(a, s, nparts);
    case NT_EPI_RESID: return dispatch_ws<NT_EPI_RESID>(a, s, nparts);
    case NT_EPI_BIAS_STATS: return dispatch_ws<NT_EPI_BIAS_STATS>(a, s, nparts);
    case NT_EPI_RESID_BN:
      return dispatch_ws<NT_EPI_RESID_BN>(a, s, nparts);
    case NT_EPI_BN_RELU: return dispatch_ws<NT_EPI_BN_RELU>(a, s, nparts);
    case NT_EPI_BN_RESID_RELU: return dispatch_ws<NT_EPI_BN_RESID_RELU>(a, s, nparts);
    case NT_EPI_BN_RESID_RELU_HEAD: return dispatch_ws<NT_EPI_BN_RESID_RELU_HEAD>(a, s, nparts);
    case NT_EPI_DROP_BN:
      return dispatch_ws<NT_EPI_DROP_BN>(a, s, nparts);
  }
  set_error("gemm_ws: bad epilogue");
  return DCNR_BAD_ARG;
}

}  // namespace dcnr
