// Fused eval deep tower (gfx950): the eval forward's whole deep tower --
// initial Linear, R ResBlocks (Linear -> BN(running stats) -> ReLU ->
// Linear -> BN -> + residual -> ReLU) and the deep head dot -- in ONE
// persistent launch whose activations never leave the chip (scoring,
// main.py:319-322; eval semantics of train.py:102-122, 161-170: dropout is
// the identity and BatchNorm uses its running statistics, so no batch-global
// barrier separates the layers).
//
//  * one 256-thread workgroup per CU, one wave per SIMD (up to 512 VGPRs);
//    each wave owns 32 samples (a tile is 128 samples per CU) and keeps their
//    activations in REGISTERS as MFMA B-operand fragments -- features on k,
//    samples on the 16 columns: h and a1 of 32 samples x 512 features are
//    256 VGPRs;
//  * the weights are the A operand.  They are streamed from L2 (4.7 MB of
//    bf16 shared by every CU) through an LDS ring by LDS-DMA, one slice
//    per step (32 output features x K, pre-packed in fragment order so each
//    wave's ds_read_b128 is one contiguous 1 KB), read by all four waves;
//  * v_mfma_f32_16x16x32_bf16: lane (g = lane/16, c = lane%16) accumulates
//    features 16b + 4g + r of sample c -- exactly what the next layer's B
//    fragment needs at elements 4(b&1) + r of k-step b/2, so a layer's output
//    is its successor's operand with no data movement; tower_pack permutes
//    the hidden weights' input columns to match (element j of lane group g in
//    k-step kt is feature 32kt + 16(j>>2) + 4g + (j&3));
//  * epilogue per slice: BN affine (Linear bias folded into the shift),
//    ReLU, the residual (read from the output registers themselves: a
//    ResBlock's second Linear overwrites h in place), bf16 pack;
//  * head: dot of the bf16 h_R with wf, 4-lane reduce, + zc (the cross half
//    of the head, written by the gather/cross kernel) + bias.
//
// HBM traffic per scored pair: the bf16 x0 row (Dp x 2 B) + zc + the logit;
// MFMA work 2 x (Dp_pad x HT + 2R x HT^2) FLOP.
#include "dcnr_internal.h"

#include <type_traits>

namespace dcnr {
namespace {

constexpr int TW_NT = 256, TW_WAVES = 4, TW_S = 32, TW_TILE = TW_WAVES * TW_S;
constexpr int TW_KT0 = 16;                    // k-steps of the initial Linear (Dp <= 512, zero padded)
constexpr int TW_SLOT = 2 * TW_KT0 * 1024 + 256;   // ring slot: 2 output blocks x 16 k-steps + constants
constexpr int TW_CONST = 2 * TW_KT0 * 1024;   // constants' offset in a slot: sc[32], sh[32]
constexpr int TW_NSLOT = 4;   // (3 slots: 636 vs 622 us per bench-size call, tools/tower_lab.sh)

typedef float f2v __attribute__((ext_vector_type(2)));
typedef bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{a, b}, bf16x2v));
}
__device__ __forceinline__ float lo16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// packed layout: the slices of layer 0 (2R+1 layers, NCH = HT/32 slices
// each), then the hidden layers', then wf [HT] fp32
__host__ __device__ inline int64_t tw_slice_bytes(int kt) { return 2048LL * kt + 256; }
__host__ __device__ inline int64_t tw_slice_off(int l, int ch, int nch, int nkt) {
  return l == 0 ? ch * tw_slice_bytes(TW_KT0)
                : nch * tw_slice_bytes(TW_KT0) + ((int64_t)(l - 1) * nch + ch) * tw_slice_bytes(nkt);
}
__host__ __device__ inline int64_t tw_packed_bytes(int R, int HT) {
  const int nch = HT / 32, nkt = HT / 32;
  return tw_slice_off(2 * R + 1, 0, nch, nkt) + (int64_t)HT * 4;
}

// --------------------------------------------------------------- pack
// One thread per 16-B weight group (8 bf16 of one lane's A fragment), then
// one per (layer, feature) for the constants, then wf.
__global__ __launch_bounds__(256) void tower_pack_kernel(TowerPack p) {
  const int HT = p.HT, nch = HT / 32, nkt = HT / 32, H = p.H;
  const int64_t g0 = (int64_t)nch * 2 * TW_KT0 * 64;   // layer 0 groups
  const int64_t gl = (int64_t)nch * 2 * nkt * 64;       // per hidden layer
  const int64_t nw = g0 + 2LL * p.R * gl;
  const int64_t nc = (int64_t)(2 * p.R + 1) * HT;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && p.err) {
#pragma unroll
    for (int e = 0; e < 64; ++e) p.err[e] = 0;
  }
  if (i < nw) {
    int l, kt_n;
    int64_t r;
    if (i < g0) { l = 0; r = i; kt_n = TW_KT0; }
    else { l = 1 + (int)((i - g0) / gl); r = (i - g0) % gl; kt_n = nkt; }
    const int lane = (int)(r % 64);
    const int kt = (int)((r / 64) % kt_n);
    const int ob = (int)((r / (64LL * kt_n)) % 2);
    const int ch = (int)(r / (128LL * kt_n));
    const int o = 32 * ch + 16 * ob + (lane & 15), g = lane >> 4;
    const float* W;
    int K;
    if (l == 0) { W = p.W0; K = p.D; }
    else { W = (l & 1) ? p.w1[(l - 1) / 2] : p.w2[(l - 1) / 2]; K = H; }
    // elements j = 0..3 and 4..7 are two runs of 4 consecutive k: two 16-B
    // loads where the row allows (K % 4 == 0, whole run inside the row)
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kh = l == 0 ? 32 * kt + 8 * g + 4 * h : 32 * kt + 16 * h + 4 * g;
      const float* src = W + (int64_t)o * K + kh;
      if (o < H && kh + 4 <= K && (K & 3) == 0) {
        const float4 f = *reinterpret_cast<const float4*>(src);
        v[4 * h] = f.x; v[4 * h + 1] = f.y; v[4 * h + 2] = f.z; v[4 * h + 3] = f.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * h + e] = (o < H && kh + e < K) ? src[e] : 0.f;
      }
    }
    uint32_t w[4];
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) w[j2] = pk2(v[2 * j2], v[2 * j2 + 1]);
    char* dst = p.out + tw_slice_off(l, ch, nch, nkt) + ((int64_t)ob * kt_n + kt) * 1024 + lane * 16;
    *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
    return;
  }
  if (i < nw + nc) {
    const int64_t r = i - nw;
    const int l = (int)(r / HT), f = (int)(r % HT);
    float sc = 0.f, sh = 0.f;
    if (f < H) {
      if (l == 0) {
        sc = 1.f;
        sh = p.b0[f];
      } else {
        const int j = (l - 1) / 2;
        const bool second = (l & 1) == 0;
        const float* b = second ? p.b2[j] : p.b1[j];
        const float* gm = second ? p.g2[j] : p.g1[j];
        const float* be = second ? p.be2[j] : p.be1[j];
        const float* rm = second ? p.rm2[j] : p.rm1[j];
        const float* rv = second ? p.rv2[j] : p.rv1[j];
        // bn_eval_multi_kernel's running-stat affine, the Linear bias folded in
        const double mean = rm[f], var = rv[f];
        const float inv = (float)(1.0 / sqrt(var + (double)BN_EPS));
        sc = gm[f] * inv;
        sh = fmaf(b[f], sc, be[f] - (float)mean * sc);
      }
    }
    const int kt_n = l == 0 ? TW_KT0 : nkt;
    float* cst = reinterpret_cast<float*>(p.out + tw_slice_off(l, f / 32, nch, nkt) + 2048LL * kt_n);
    cst[f % 32] = sc;
    cst[32 + f % 32] = sh;
    return;
  }
  if (i < nw + nc + HT) {
    const int f = (int)(i - nw - nc);
    reinterpret_cast<float*>(p.out + tw_slice_off(2 * p.R + 1, 0, nch, nkt))[f] = f < H ? p.wf[f] : 0.f;
  }
}

// ----------------------------------------------------------- one slice
// A slice's accumulators and its 32 features' BN constants, kept in
// registers until its epilogue runs inside the NEXT slice's k-loop (beside
// that slice's MFMAs: one wave per SIMD has no partner to hide a separate
// epilogue phase behind).
struct Pend {
  f32x4 acc[2][2];   // [output block][sample block]
  float4 sc[2], sh[2];
};

// MODE 0: initial Linear (acc + b0), 1: BN + ReLU, 2: BN + residual + ReLU
// (the residual is the output fragment itself).  Piece p of 8 finishes two
// features (r = 2(p&1), +1) of output block p>>2 for sample block (p>>1)&1.
template <int MODE>
__device__ __forceinline__ void epi_piece(const Pend& pd, int p, u32x4& w0, u32x4& w1) {
  const int ob = p >> 2, sb = (p >> 1) & 1, hf = p & 1;
  u32x4& w = sb ? w1 : w0;
  const f32x4& ac = pd.acc[ob][sb];
  float v0 = fmaf(ac[2 * hf], hf ? pd.sc[ob].z : pd.sc[ob].x, hf ? pd.sh[ob].z : pd.sh[ob].x);
  float v1 = fmaf(ac[2 * hf + 1], hf ? pd.sc[ob].w : pd.sc[ob].y, hf ? pd.sh[ob].w : pd.sh[ob].y);
  if constexpr (MODE == 2) {
    const uint32_t r = w[2 * ob + hf];
    v0 += lo16(r);
    v1 += hi16(r);
  }
  if constexpr (MODE >= 1) {
    // ReLU on the packed pair: bf16 rounding keeps the sign, so
    // max(bf16(v), 0) as two int16 lanes (v_pk_max_i16: negatives and -0
    // -> +0) is bf16(max(v, 0)) -- one instruction instead of two v_max_f32
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    const s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(s16x2, pk2(v0, v1)), s16x2{0, 0});
    w[2 * ob + hf] = __builtin_bit_cast(uint32_t, r);
  } else {
    w[2 * ob + hf] = pk2(v0, v1);
  }
}

// One slice (step): the k-loop of 2 output blocks x 2 sample blocks into
// `cur`, with the previous slice's epilogue (`pend`, PEND) in its first 8
// k-steps and the next slice's LDS-DMA pieces on its odd ones; then the
// slice's constants into `cur`.  p0/p1: the previous
// slice's output fragments.
template <int KT, int MODE, bool PEND, class Dma>
__device__ __forceinline__ void tw_slice(const char* sl, int g, int lane, const u32x4 (&in)[16][2],
                                         Pend& cur, const Pend& pend, u32x4& p0, u32x4& p1,
                                         const Dma& dma) {
#pragma unroll
  for (int ob = 0; ob < 2; ++ob)
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) cur.acc[ob][sb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* ab = sl + lane * 16;
  auto rd = [&](int ob, int kt) { return *reinterpret_cast<const bf16x8*>(ab + (ob * KT + kt) * 1024); };
  bf16x8 af[3][2];   // A fragments two k-steps ahead (one ahead: +2.5 % per call)
  af[0][0] = rd(0, 0);
  af[0][1] = rd(1, 0);
  if (KT > 1) { af[1][0] = rd(0, 1); af[1][1] = rd(1, 1); }
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 2 < KT) {
      af[(kt + 2) % 3][0] = rd(0, kt + 2);
      af[(kt + 2) % 3][1] = rd(1, kt + 2);
    }
    // the DMA pieces on odd k-steps, so they spread over the whole slice
    // (issue-bound at one wave per SIMD: on k-steps 0..8 beside the epilogue
    // pieces 2-3 % slower, profiles/lab/r05_tower_ablation.txt)
    if (kt & 1) dma(kt >> 1);
#pragma unroll
    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
        cur.acc[ob][sb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            af[kt % 3][ob], __builtin_bit_cast(bf16x8, in[kt][sb]), cur.acc[ob][sb], 0, 0, 0);
    const bool piece = PEND && kt < 8;
    if (piece) epi_piece<MODE>(pend, kt, p0, p1);
    if (kt + 2 < KT) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS reads two steps ahead
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);               // an MFMA
      if (piece) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // ... then epilogue VALU
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // (short k-loops: the DMA and epilogue pieces left over)
  for (int d = KT / 2; d <= TW_KT0 / 2; ++d) dma(d);
  if constexpr (PEND) {
#pragma unroll
    for (int p = KT; p < 8; ++p) epi_piece<MODE>(pend, p, p0, p1);
  }
  const float* cst = reinterpret_cast<const float*>(sl + TW_CONST);
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    cur.sc[ob] = *reinterpret_cast<const float4*>(cst + 16 * ob + 4 * g);
    cur.sh[ob] = *reinterpret_cast<const float4*>(cst + 32 + 16 * ob + 4 * g);
  }
  // pin the finished epilogue here: left alone, the compiler sinks it to the
  // next layer's first use and keeps every slice's accumulators alive
  if constexpr (PEND) asm volatile("" : "+a"(p0), "+a"(p1));
}

// the whole epilogue of a layer's last slice, right after its k-loop
template <int MODE>
__device__ __forceinline__ void tw_finish(const Pend& pd, u32x4& o0, u32x4& o1) {
#pragma unroll
  for (int p = 0; p < 8; ++p) epi_piece<MODE>(pd, p, o0, o1);
  asm volatile("" : "+a"(o0), "+a"(o1));
}

template <int NKT>
__global__ __launch_bounds__(TW_NT, 1) void tower_kernel(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int NCH = NKT;   // 32-feature slices per layer (HT / 32)
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* wf_s = reinterpret_cast<float*>(lds + TW_NSLOT * TW_SLOT);
  const u32x4 wr = rsrc_words(a.wp, a.wp_bytes);
  const uint32_t lbase = lds_addr(lds);
  const int per_tile = NCH * (1 + 2 * a.R);
  const int my_tiles = a.ntiles > (int)blockIdx.x ? (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int total = my_tiles * per_tile;
  // the slice stream (the same sequence of layers for every tile): step q
  // consumes slice q in slot q % NSLOT, and issues slice q + NSLOT - 1.  The
  // issue cursor (layer, slice, byte offset, slot) advances by additions
  // only: this code is inlined at every step of the unrolled layers.
  int i_layer = 0, i_ch = 0, i_off = 0, i_slot = 0, i_left = total;
  // the slice being issued during this step: LDS slot, source offset (an
  // out-of-range one past the end of the stream: the DMAs then write zeros
  // into a slot nobody reads again), 1-KB pieces per wave
  uint32_t i_dst = 0;
  int i_src = 0, i_pcs = 0;
  auto issue_begin = [&]() {
    i_dst = __builtin_amdgcn_readfirstlane(lbase + i_slot * TW_SLOT);
    i_src = i_left > 0 ? i_off : 0x7f000000;
    i_pcs = (i_layer == 0 ? TW_KT0 : NKT) / 2;
    if (i_left > 0) {
      --i_left;
      i_off += (i_layer == 0 ? TW_KT0 : NKT) * 2048 + 256;
      if (++i_ch == NCH) {
        i_ch = 0;
        if (++i_layer == 2 * a.R + 1) { i_layer = 0; i_off = 0; }
      }
    }
    i_slot = i_slot + 1 == TW_NSLOT ? 0 : i_slot + 1;
  };
  // piece d of the slice being issued (d == pieces: its constants), one per
  // odd k-step of the consuming slice: each LDS-DMA's issue cost then sits
  // beside MFMAs instead of in a burst after the barrier
  auto issue_piece = [&](int d) {
    const int pcs = NKT == TW_KT0 ? TW_KT0 / 2 : i_pcs;
    if (d < pcs) {
      const int pc = wave * pcs + d;
      dma16s(wr, lane * 16, __builtin_amdgcn_readfirstlane(i_src + pc * 1024), i_dst + pc * 1024);
    } else if (d == pcs) {
      if (lane < 4)
        dma16s(wr, lane * 16, __builtin_amdgcn_readfirstlane(i_src + pcs * 4096 + wave * 64),
               i_dst + TW_CONST + wave * 64);
    }
  };
  auto issue = [&]() {   // a whole slice at once (the prologue)
    issue_begin();
    for (int d = 0; d <= i_pcs; ++d) issue_piece(d);
  };
  // every wave's DMAs of slice q landed, and every wave is done with slot
  // (q - 1) % NSLOT, which slice q + NSLOT - 1 then refills (the younger
  // DMAs in flight at the wait: those of the NSLOT - 2 slices after q,
  // NKT/2 + 1 or more per wave and slice; near the end of the stream fewer)
  auto sync = [&](int q) {
    constexpr int PER = NKT / 2 + 1;
    if (q + TW_NSLOT - 2 < total)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((TW_NSLOT - 2) * PER) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue_begin();
  };
  // the call's id-check word (the gather before this launch set it) to its
  // mirror, e.g. pinned host memory: no copy of its own on the stream
  if (a.err_mirror && blockIdx.x == 0 && tid == 0)
    __hip_atomic_store(a.err_mirror, *a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int f = tid; f < NKT * 32; f += TW_NT)
    wf_s[f] = reinterpret_cast<const float*>(a.wp + tw_slice_off(2 * a.R + 1, 0, NCH, NKT))[f];
  for (int p = 0; p < TW_NSLOT - 1; ++p) issue();

  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x0, a.M * a.ldx * 2);
  u32x4 X[16][2], H[16][2];
  Pend pa, pb;
  int q = 0, c_slot = 0;   // step, and the slot it reads
  for (int t = 0; t < my_tiles; ++t) {
    const int64_t s0 = ((int64_t)blockIdx.x + (int64_t)t * gridDim.x) * TW_TILE + wave * TW_S;
    // x0 fragments in natural k order: X[kt][sb] = x0[s0 + 16sb + c][32kt + 8g .. +7]
#pragma unroll
    for (int kt = 0; kt < TW_KT0; ++kt)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int64_t s = s0 + 16 * sb + c;
        const int k = 32 * kt + 8 * g;
        X[kt][sb] = __builtin_amdgcn_raw_buffer_load_b128(
            xr, (s < a.M && k < a.Dp) ? (int)((s * a.ldx + k) * 2) : OOR, 0, 0);
      }
    // one layer: NCH slices, slice ch's epilogue inside slice ch+1's k-loop,
    // the last one's right after its own
    auto layer = [&](auto kt_c, auto mode_c, const u32x4 (&in)[16][2], u32x4 (&out)[16][2]) {
      constexpr int KT = decltype(kt_c)::value, MODE = decltype(mode_c)::value;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch, ++q) {
        sync(q);
        const char* sl = lds + c_slot * TW_SLOT;
        c_slot = c_slot + 1 == TW_NSLOT ? 0 : c_slot + 1;
        Pend& cur = (ch & 1) ? pb : pa;
        const Pend& prev = (ch & 1) ? pa : pb;
        if (ch == 0) tw_slice<KT, MODE, false>(sl, g, lane, in, cur, prev, out[0][0], out[0][1], issue_piece);
        else tw_slice<KT, MODE, true>(sl, g, lane, in, cur, prev, out[ch - 1][0], out[ch - 1][1], issue_piece);
      }
      tw_finish<MODE>((NCH & 1) ? pa : pb, out[NCH - 1][0], out[NCH - 1][1]);
    };
    using KT0c = std::integral_constant<int, TW_KT0>;
    using NKTc = std::integral_constant<int, NKT>;
    layer(KT0c{}, std::integral_constant<int, 0>{}, X, H);       // initial Linear: X -> H
    for (int j = 0; j < a.R; ++j) {
      layer(NKTc{}, std::integral_constant<int, 1>{}, H, X);     // a1 = relu(BN1(h W1^T + b1))
      layer(NKTc{}, std::integral_constant<int, 2>{}, X, H);     // h = relu(BN2(a1 W2^T + b2) + h)
    }
    // deep head: sum_f bf16(h_R[f]) wf[f], this lane's features, then the
    // sample's four lanes (g = 0..3): half-wave swap, then row swap
    float z[2] = {0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const float4 wa = *reinterpret_cast<const float4*>(wf_s + 32 * kt + 4 * g);
      const float4 wb = *reinterpret_cast<const float4*>(wf_s + 32 * kt + 16 + 4 * g);
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const u32x4 h = H[kt][sb];
        z[sb] = fmaf(lo16(h[0]), wa.x, z[sb]);
        z[sb] = fmaf(hi16(h[0]), wa.y, z[sb]);
        z[sb] = fmaf(lo16(h[1]), wa.z, z[sb]);
        z[sb] = fmaf(hi16(h[1]), wa.w, z[sb]);
        z[sb] = fmaf(lo16(h[2]), wb.x, z[sb]);
        z[sb] = fmaf(hi16(h[2]), wb.y, z[sb]);
        z[sb] = fmaf(lo16(h[3]), wb.z, z[sb]);
        z[sb] = fmaf(hi16(h[3]), wb.w, z[sb]);
      }
    }
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const unsigned u = __float_as_uint(z[sb]);
      auto h2 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
      const float t2 = __uint_as_float(h2[0]) + __uint_as_float(h2[1]);
      const unsigned ut = __float_as_uint(t2);
      auto h4 = __builtin_amdgcn_permlane16_swap(ut, ut, false, false);
      const float zs = __uint_as_float(h4[0]) + __uint_as_float(h4[1]);
      const int64_t s = s0 + 16 * sb + c;
      if (g == 0 && s < a.M) a.logits[s] = zs + a.zc[s] + a.bias[0];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool tower_supported(int Dp, int H, int R) {
  return Dp <= 512 && H >= 1 && rup(H, 64) <= 512 && R >= 1 && R <= MAX_RES_TW;
}
int64_t tower_ws_bytes(int H, int R) { return tw_packed_bytes(R, (int)rup(H, 64)); }

dcnr_status tower_pack(const TowerPack& p0, hipStream_t s) {
  TowerPack p = p0;
  p.HT = (int)rup(p.H, 64);
  const int nch = p.HT / 32;
  const int64_t n = (int64_t)nch * 2 * TW_KT0 * 64 + 2LL * p.R * nch * 2 * (p.HT / 32) * 64 +
                    (int64_t)(2 * p.R + 1) * p.HT + p.HT;
  hipLaunchKernelGGL(tower_pack_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, p);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status eval_tower(const TowerArgs& a0, hipStream_t s) {
  TowerArgs a = a0;
  const int HT = (int)rup(a.H, 64), nkt = HT / 32;
  if (!tower_supported(a.Dp, a.H, a.R) || a.ldx < a.Dp || a.ldx % 8) {
    set_error("eval_tower: unsupported Dp=%d H=%d R=%d", a.Dp, a.H, a.R);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  a.wp_bytes = tw_packed_bytes(a.R, HT);
  const size_t lds = TW_NSLOT * TW_SLOT + (size_t)HT * 4;
  const void* k = nullptr;
  switch (nkt) {
    case 2: k = (const void*)tower_kernel<2>; break;
    case 4: k = (const void*)tower_kernel<4>; break;
    case 6: k = (const void*)tower_kernel<6>; break;
    case 8: k = (const void*)tower_kernel<8>; break;
    case 10: k = (const void*)tower_kernel<10>; break;
    case 12: k = (const void*)tower_kernel<12>; break;
    case 14: k = (const void*)tower_kernel<14>; break;
    case 16: k = (const void*)tower_kernel<16>; break;
  }
  TRY_ST(set_max_dyn_lds(k, lds));
  // 32-bit buffer offsets into x0: launches of < 2^31 bytes of rows
  const int64_t chunk = std::max<int64_t>(TW_TILE, ((int64_t(1) << 31) - 1) / (a.ldx * 2) / TW_TILE * TW_TILE);
  for (int64_t m0 = 0; m0 < a0.M; m0 += chunk) {
    TowerArgs b = a;
    b.M = std::min(chunk, a0.M - m0);
    b.x0 = a.x0 + m0 * a.ldx;
    b.zc = a.zc + m0;
    b.logits = a.logits + m0;
    b.ntiles = (int)cdiv(b.M, TW_TILE);
    // the mirror is stored once, by the last chunk: an earlier chunk's store
    // would let the host recycle the slot while a later one can still write it
    b.err_mirror = m0 + b.M >= a0.M ? a.err_mirror : nullptr;
    const int grid = (int)std::min<int64_t>(b.ntiles, 256);
    void* args[] = {&b};
    DCNR_HIP(hipLaunchKernel(k, dim3(grid), dim3(TW_NT), args, lds, s));
  }
  return DCNR_OK;
}

}  // namespace dcnr
