// LAB (not built into libdcnr): the fused eval tower on v_mfma_f32_32x32x16_bf16,
// measured 5 % slower than csrc/tower.hip (profiles/lab/r05_tower_ablation.txt).
// Build as a replacement of tower.o (tools/lab/r05_m32.sh, -mllvm -amdgpu-mfma-vgpr-form).
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
constexpr int TW_KT0 = 32;                    // 16-deep k-steps of the initial Linear (Dp <= 512, zero padded)
constexpr int TW_SLOT = TW_KT0 * 1024 + 256;  // ring slot: 32 output features x 32 k-steps + constants
constexpr int TW_CONST = TW_KT0 * 1024;       // constants' offset in a slot: sc[32], sh[32]
constexpr int TW_NSLOT = 4;   // (3 slots: 636 vs 622 us per bench-size call, tools/tower_lab.sh)
constexpr int TW_AHEAD = 3;   // A fragments read this many k-steps ahead

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{a, b}, bf16x2v));
}
__device__ __forceinline__ float lo16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// v_mfma_f32_32x32x16_bf16 (32 output features x 32 samples x 16 k): lane
// (h = lane / 32, c = lane % 32) accumulates features (r & 3) + 8 (r >> 2) +
// 4h of sample c in register r.  Registers 8s .. 8s + 7 are then exactly the
// next layer's B fragment of k-step 2 ch + s (element j = register 8s + j),
// provided the next layer's weights take their input columns in that order:
// element j of lane half h in k-step kt is feature
//   32 (kt >> 1) + 16 (kt & 1) + 8 (j >> 2) + 4h + (j & 3)
// (hidden layers; the initial Linear reads x0 in natural order, 16 kt + 8h + j).
__host__ __device__ inline int tw_hidden_col(int kt, int h, int j) {
  return 32 * (kt >> 1) + 16 * (kt & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}

// packed layout: the slices of layer 0 (2R+1 layers, NCH = HT/32 slices
// each, a slice = 32 output features x all k-steps, 1 KB per k-step), then
// the hidden layers', then wf [HT] fp32
__host__ __device__ inline int64_t tw_slice_bytes(int kt) { return 1024LL * kt + 256; }
__host__ __device__ inline int64_t tw_slice_off(int l, int ch, int nch, int nkt) {
  return l == 0 ? ch * tw_slice_bytes(TW_KT0)
                : nch * tw_slice_bytes(TW_KT0) + ((int64_t)(l - 1) * nch + ch) * tw_slice_bytes(nkt);
}
__host__ __device__ inline int64_t tw_packed_bytes(int R, int HT) {
  const int nch = HT / 32, nkt = HT / 16;
  return tw_slice_off(2 * R + 1, 0, nch, nkt) + (int64_t)HT * 4;
}

// --------------------------------------------------------------- pack
// One thread per 16-B weight group (8 bf16 of one lane's A fragment), then
// one per (layer, feature) for the constants, then wf.
__global__ __launch_bounds__(256) void tower_pack_kernel(TowerPack p) {
  const int HT = p.HT, nch = HT / 32, nkt = HT / 16, H = p.H;
  const int64_t g0 = (int64_t)nch * TW_KT0 * 64;   // layer 0 groups
  const int64_t gl = (int64_t)nch * nkt * 64;       // per hidden layer
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
    const int ch = (int)(r / (64LL * kt_n));
    const int o = 32 * ch + (lane & 31), h = lane >> 5;
    const float* W;
    int K;
    if (l == 0) { W = p.W0; K = p.D; }
    else { W = (l & 1) ? p.w1[(l - 1) / 2] : p.w2[(l - 1) / 2]; K = H; }
    // elements j = 0..3 and 4..7 are two runs of 4 consecutive k: two 16-B
    // loads where the row allows (K % 4 == 0, whole run inside the row)
    float v[8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int kh = l == 0 ? 16 * kt + 8 * h + 4 * q : tw_hidden_col(kt, h, 4 * q);
      const float* src = W + (int64_t)o * K + kh;
      if (o < H && kh + 4 <= K && (K & 3) == 0) {
        const float4 f = *reinterpret_cast<const float4*>(src);
        v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = (o < H && kh + e < K) ? src[e] : 0.f;
      }
    }
    uint32_t w[4];
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) w[j2] = pk2(v[2 * j2], v[2 * j2 + 1]);
    char* dst = p.out + tw_slice_off(l, ch, nch, nkt) + (int64_t)kt * 1024 + lane * 16;
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
    float* cst = reinterpret_cast<float*>(p.out + tw_slice_off(l, f / 32, nch, nkt) + 1024LL * kt_n);
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
// A slice's accumulators and its features' BN constants (this lane's 16
// features: sc[q] / sh[q] hold registers 4q .. 4q + 3), kept until its
// epilogue runs inside the NEXT slice's k-loop (beside that slice's MFMAs:
// one wave per SIMD has no partner to hide a separate epilogue phase behind).
struct Pend {
  f32x16 acc;
  float4 sc[4], sh[4];
};

// MODE 0: initial Linear (acc + b0), 1: BN + ReLU, 2: BN + residual + ReLU
// (the residual is the output fragment itself).  Piece p of 8 finishes
// registers 2p, 2p + 1: word p & 3 of output fragment p >> 2.
template <int MODE>
__device__ __forceinline__ void epi_piece(const Pend& pd, int p, u32x4& w0, u32x4& w1) {
  const int q = p >> 1, e = 2 * (p & 1);
  u32x4& w = (p >> 2) ? w1 : w0;
  const float4 sc = pd.sc[q], sh = pd.sh[q];
  float v0 = fmaf(pd.acc[2 * p], e ? sc.z : sc.x, e ? sh.z : sh.x);
  float v1 = fmaf(pd.acc[2 * p + 1], e ? sc.w : sc.y, e ? sh.w : sh.y);
  if constexpr (MODE == 2) {
    const uint32_t r = w[p & 3];
    v0 += lo16(r);
    v1 += hi16(r);
  }
  if constexpr (MODE >= 1) {
    v0 = fmaxf(v0, 0.f);
    v1 = fmaxf(v1, 0.f);
  }
  w[p & 3] = pk2(v0, v1);
}

// One slice (step): the k-loop of 32 features x 32 samples into `cur`, with
// the previous slice's epilogue (`pend`, PEND) on its odd k-steps and this
// step's LDS-DMA pieces on every fourth; then the slice's constants into
// `cur`.  p0/p1: the previous slice's output fragments.
template <int KT, int MODE, bool PEND, class Dma>
__device__ __forceinline__ void tw_slice(const char* sl, int h, int lane, const u32x4 (&in)[TW_KT0],
                                         Pend& cur, const Pend& pend, u32x4& p0, u32x4& p1,
                                         const Dma& dma) {
#pragma unroll
  for (int r = 0; r < 16; ++r) cur.acc[r] = 0.f;
  const char* ab = sl + lane * 16;
  auto rd = [&](int kt) { return *reinterpret_cast<const bf16x8*>(ab + kt * 1024); };
  constexpr int NA = TW_AHEAD + 1;
  bf16x8 af[NA];
#pragma unroll
  for (int kt = 0; kt < TW_AHEAD && kt < KT; ++kt) af[kt] = rd(kt);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + TW_AHEAD < KT) af[(kt + TW_AHEAD) % NA] = rd(kt + TW_AHEAD);
    if ((kt & 3) == 0) dma(kt >> 2);
    cur.acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kt % NA], __builtin_bit_cast(bf16x8, in[kt]), cur.acc,
                                                      0, 0, 0);
    if (PEND && (kt & 1) && kt < 16) epi_piece<MODE>(pend, kt >> 1, p0, p1);
    __builtin_amdgcn_sched_barrier(0);
  }
  // (short k-loops: the DMA and epilogue pieces left over)
  for (int d = (KT + 3) / 4; d <= TW_KT0 / 4; ++d) dma(d);
  if constexpr (PEND) {
#pragma unroll
    for (int p = KT / 2; p < 8; ++p) epi_piece<MODE>(pend, p, p0, p1);
  }
  const float* cst = reinterpret_cast<const float*>(sl + TW_CONST);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    cur.sc[q] = *reinterpret_cast<const float4*>(cst + 8 * q + 4 * h);
    cur.sh[q] = *reinterpret_cast<const float4*>(cst + 32 + 8 * q + 4 * h);
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

template <int NCH>
__global__ __launch_bounds__(TW_NT, 1) void tower_kernel(TowerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int NKT = 2 * NCH;   // 16-deep k-steps of a hidden layer (HT / 16); NCH 32-feature slices
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
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
  // into a slot nobody reads again), 1-KB pieces (k-steps) per wave
  uint32_t i_dst = 0;
  int i_src = 0, i_pcs = 0;
  auto issue_begin = [&]() {
    i_dst = __builtin_amdgcn_readfirstlane(lbase + i_slot * TW_SLOT);
    i_src = i_left > 0 ? i_off : 0x7f000000;
    i_pcs = (i_layer == 0 ? TW_KT0 : NKT) / 4;
    if (i_left > 0) {
      --i_left;
      i_off += (i_layer == 0 ? TW_KT0 : NKT) * 1024 + 256;
      if (++i_ch == NCH) {
        i_ch = 0;
        if (++i_layer == 2 * a.R + 1) { i_layer = 0; i_off = 0; }
      }
    }
    i_slot = i_slot + 1 == TW_NSLOT ? 0 : i_slot + 1;
  };
  // piece d of the slice being issued (d == pieces: its constants), one per
  // four k-steps of the consuming slice: each LDS-DMA's issue cost then sits
  // beside MFMAs instead of in a burst after the barrier
  auto issue_piece = [&](int d) {
    const int pcs = NKT == TW_KT0 ? TW_KT0 / 4 : i_pcs;
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
  // NKT/4 + 1 or more per wave and slice; near the end of the stream fewer)
  auto sync = [&](int q) {
    constexpr int PER = NKT / 4 + 1;
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
  for (int f = tid; f < NCH * 32; f += TW_NT)
    wf_s[f] = reinterpret_cast<const float*>(a.wp + tw_slice_off(2 * a.R + 1, 0, NCH, NKT))[f];
  for (int p = 0; p < TW_NSLOT - 1; ++p) issue();

  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x0, a.M * a.ldx * 2);
  u32x4 X[TW_KT0], H[TW_KT0];
  Pend pa, pb;
  int q = 0, c_slot = 0;   // step, and the slot it reads
  for (int t = 0; t < my_tiles; ++t) {
    const int64_t s0 = ((int64_t)blockIdx.x + (int64_t)t * gridDim.x) * TW_TILE + wave * TW_S;
    const int64_t s = s0 + c;
    // x0 fragments in natural k order: X[kt] = x0[s][16kt + 8h .. +7]
#pragma unroll
    for (int kt = 0; kt < TW_KT0; ++kt) {
      const int k = 16 * kt + 8 * h;
      X[kt] = __builtin_amdgcn_raw_buffer_load_b128(xr, (s < a.M && k < a.Dp) ? (int)((s * a.ldx + k) * 2) : OOR,
                                                   0, 0);
    }
    // one layer: NCH slices, slice ch's epilogue inside slice ch+1's k-loop,
    // the last one's right after its own
    auto layer = [&](auto kt_c, auto mode_c, const u32x4 (&in)[TW_KT0], u32x4 (&out)[TW_KT0]) {
      constexpr int KT = decltype(kt_c)::value, MODE = decltype(mode_c)::value;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch, ++q) {
        sync(q);
        const char* sl = lds + c_slot * TW_SLOT;
        c_slot = c_slot + 1 == TW_NSLOT ? 0 : c_slot + 1;
        Pend& cur = (ch & 1) ? pb : pa;
        const Pend& prev = (ch & 1) ? pa : pb;
        if (ch == 0) tw_slice<KT, MODE, false>(sl, h, lane, in, cur, prev, out[0], out[1], issue_piece);
        else tw_slice<KT, MODE, true>(sl, h, lane, in, cur, prev, out[2 * ch - 2], out[2 * ch - 1], issue_piece);
      }
      tw_finish<MODE>((NCH & 1) ? pa : pb, out[2 * NCH - 2], out[2 * NCH - 1]);
    };
    using KT0c = std::integral_constant<int, TW_KT0>;
    using NKTc = std::integral_constant<int, NKT>;
    layer(KT0c{}, std::integral_constant<int, 0>{}, X, H);       // initial Linear: X -> H
    for (int j = 0; j < a.R; ++j) {
      layer(NKTc{}, std::integral_constant<int, 1>{}, H, X);     // a1 = relu(BN1(h W1^T + b1))
      layer(NKTc{}, std::integral_constant<int, 2>{}, X, H);     // h = relu(BN2(a1 W2^T + b2) + h)
    }
    // deep head: sum_f bf16(h_R[f]) wf[f] over this lane's features, then
    // the sample's two lanes (h = 0, 1)
    float z = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const float4 wa = *reinterpret_cast<const float4*>(wf_s + tw_hidden_col(kt, h, 0));
      const float4 wb = *reinterpret_cast<const float4*>(wf_s + tw_hidden_col(kt, h, 4));
      const u32x4 hv = H[kt];
      z = fmaf(lo16(hv[0]), wa.x, z);
      z = fmaf(hi16(hv[0]), wa.y, z);
      z = fmaf(lo16(hv[1]), wa.z, z);
      z = fmaf(hi16(hv[1]), wa.w, z);
      z = fmaf(lo16(hv[2]), wb.x, z);
      z = fmaf(hi16(hv[2]), wb.y, z);
      z = fmaf(lo16(hv[3]), wb.z, z);
      z = fmaf(hi16(hv[3]), wb.w, z);
    }
    const unsigned u = __float_as_uint(z);
    auto h2 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    const float zs = __uint_as_float(h2[0]) + __uint_as_float(h2[1]);
    if (h == 0 && s < a.M) a.logits[s] = zs + a.zc[s] + a.bias[0];
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
  const int64_t n = (int64_t)nch * TW_KT0 * 64 + 2LL * p.R * nch * (p.HT / 16) * 64 +
                    (int64_t)(2 * p.R + 1) * p.HT + p.HT;
  hipLaunchKernelGGL(tower_pack_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, p);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

dcnr_status eval_tower(const TowerArgs& a0, hipStream_t s) {
  TowerArgs a = a0;
  const int HT = (int)rup(a.H, 64), nkt = HT / 32;   // 32-feature slices per layer
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
