// Pipelined weight-stationary GEMM for the bf16 deep tower's train forward
// (gfx950): the initial Linear and both Linears of every ResBlock
// (train.py:143, 105, 109 under :161-165),
//
//   C[M, N] = X[M, K] . W[N, K]^T + bias  (bf16 out),  256 < K <= 512,
//   optionally with the BatchNorm-statistics epilogue
//   part = [sum(c - bias), sum((c - bias)^2)] over the stored bf16 c.
//
// gemm_ws.hip's layout (W resident in registers, X tiles staged through LDS
// by LDS-DMA and read by every wave as MFMA B fragments) with one wave per
// SIMD instead of two, so nothing on the SIMD hides a separate epilogue
// phase; instead the epilogue of tile i-1 runs INSIDE tile i's k-loop:
//  * a workgroup owns a 256-column slice of W; each of its 4 waves keeps 64
//    columns x K resident as A fragments (256 AGPRs), so every X fragment
//    read from LDS feeds 8 MFMAs (gemm_ws: 4) -- half the LDS reads per
//    FLOP;
//  * X tiles of 32 rows (32 KB) stream through a 4-buffer LDS ring, one tile
//    ahead of the one being consumed besides the next (DMA pieces issued one
//    per k-step in the first half of each tile);
//  * two accumulator sets: tile i accumulates into one while tile i-1's
//    bias add, bf16 pack, statistics and 16-B row stores are spread over the
//    k-steps between the MFMAs (1-2 VALU per MFMA gap);
//  * one barrier per tile, two k-steps before its end, after which the next
//    tile's first fragments are read: no exposed LDS latency at tile starts.
//
// The C stores use a per-tile buffer descriptor and a constant 0 soffset,
// never an SGPR soffset: hipcc's hazard recognizer (ROCm 7.2) leaves out the
// two wait states a >64-bit MUBUF store needs before its data VGPRs are
// rewritten when the store has a REGISTER soffset, and the round-5 version
// of this kernel (soffset = the tile's row offset) then stored the next
// values of 4 lanes of one 16-B store now and then, whenever the memory
// pipeline was backed up.
#include "dcnr_internal.h"

namespace dcnr {
namespace {

constexpr int WP_NT = 256, WP_WAVES = 4, WP_WC = 64, WP_TN = WP_WAVES * WP_WC;
constexpr int WP_TM = 32, WP_KT = 16, WP_P = 1024, WP_TILE = WP_TM * WP_P;
constexpr int WP_NB = 4;                       // X-tile buffers in the LDS ring
constexpr int WP_DPW = WP_TM / WP_WAVES;       // 1-KB DMA pieces (rows) per wave per tile
constexpr size_t WP_LDS = (size_t)WP_NB * WP_TILE;
static_assert(WP_LDS <= 160 * 1024, "LDS budget");

typedef float f2v __attribute__((ext_vector_type(2)));
typedef bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2v{a, b}, bf16x2v));
}
__device__ __forceinline__ f2v unpack2(uint32_t w) {
  return f2v{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
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

// STATS: the BatchNorm-statistics epilogue; TAIL: the last tile may be
// partial (M % 32 != 0), rows past M left out of the statistics.
template <bool STATS, bool TAIL>
__global__ __launch_bounds__(WP_NT, 1) void gemm_wsp_kernel(NtArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, l15 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nsl = a.nslices, bid = blockIdx.x;
  const int slice = (bid / 8) % nsl;                        // both slices of a group on one XCD
  const int group = (bid % 8) + 8 * (bid / (8 * nsl));
  const int groups = a.groups;
  const int nw = slice * WP_TN + wave * WP_WC;               // this wave's first column
  const int ntl = a.mtiles > group ? (int)((a.mtiles - 1 - group) / groups + 1) : 0;
  const uint32_t lbase = lds_addr(lds);

  // ---- X-tile DMA: piece d of a tile is row r = wave*8 + d (1 KB); lane
  // reads chunk c = lane ^ (r & 15) (lands at position c ^ (r & 15) =
  // lane).  Per lane and piece the chunk offset is fixed (voff[d]); the row
  // offset is the SGPR soffset; the descriptor and destination are set once
  // per tile.  Past the last tile: an empty descriptor (zeros into a buffer
  // no wave reads again), so every k-loop issues the same number of DMAs.
  int voff[WP_DPW];
#pragma unroll
  for (int d = 0; d < WP_DPW; ++d) {
    const int c = lane ^ ((wave * WP_DPW + d) & 15);
    voff[d] = c * 8 < a.K ? c * 16 : OOR;
  }
  const int rstride = (int)(a.ldx * 2);                      // bytes per X row
  const int rbase = wave * WP_DPW * rstride;
  struct TileDma { u32x4 rs; uint32_t dst; };
  auto tile_dma = [&](int i) {
    const bool live = i < ntl;
    const int64_t m0 = (group + (int64_t)(live ? i : 0) * groups) * WP_TM;
    const int64_t rows = live ? a.M - m0 : 0;
    TileDma t;
    t.rs = rsrc_words(a.X + m0 * a.ldx, rows > 0 ? rows * a.ldx * 2 : 0);
    t.dst = lbase + (uint32_t)((i & (WP_NB - 1)) * WP_TILE + wave * WP_DPW * WP_P);
    return t;
  };
  auto piece = [&](const TileDma& t, int d) {
    dma16s(t.rs, voff[d], rbase + d * rstride, t.dst + d * WP_P);
  };
  {
    const TileDma t0 = tile_dma(0), t1 = tile_dma(1);
#pragma unroll
    for (int d = 0; d < WP_DPW; ++d) piece(t0, d);
#pragma unroll
    for (int d = 0; d < WP_DPW; ++d) piece(t1, d);
  }

  // resident W: A fragments (column block cb, k-step kt) of columns
  // nw + 16cb + l15, k = 32kt + 8q .. +7, held in AGPRs for the whole launch
  bf16x8 wf[4][WP_KT];
  {
    const __amdgpu_buffer_rsrc_t wr = buf_rsrc(a.W, (int64_t)a.N * a.ldw * 2);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int n = nw + cb * 16 + l15;
#pragma unroll
      for (int kt = 0; kt < WP_KT; ++kt) {
        const int k = kt * 32 + 8 * q;
        const bool ok = n < a.N && k < a.K;
        wf[cb][kt] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, ok ? (int)(((int64_t)n * a.ldw + k) * 2) : OOR, 0, 0));
      }
    }
  }
  // bias of this lane's accumulator columns nw + 16cb + 4q .. +3
  float bias[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int n = nw + cb * 16 + q * 4;
    const bool ok = a.bias && n < a.N;   // (N % 8 == 0: all four columns)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[cb][r] = ok ? a.bias[n + r] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int kt = 0; kt < WP_KT; ++kt) asm volatile("" : "+a"(wf[cb][kt]));
  __syncthreads();

  // per-lane column partials [sum, sum2][cb][column r], over all tiles
  float st[2][4][4];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[k][cb][r] = 0.f;

  // fragment (kt, rb): row rb*16 + l15, physical chunk (4kt + q) ^ l15
  const uint32_t rowoff = (uint32_t)l15 * WP_P;
  int coff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) coff[j] = ((4 * j + q) ^ l15) * 16;
  auto xrd = [&](const char* xb, int kt, int rb) {
    return *reinterpret_cast<const bf16x8*>(xb + rb * 16 * WP_P + (kt >> 2) * 256 + coff[kt & 3]);
  };
  const int nst = nw + (q & 1) * 16 + (q >> 1) * 8;          // store-layout column (pair 0)
  // epilogue piece e (0..15) of the tile at row mp: row block e >> 3, column
  // block (e >> 1) & 3, column pair e & 1 -> its packed bf16 word ow[cb][d];
  // after a row block's last piece, its two 16-B row stores (epi_store)
  uint32_t ow[4][2];
  auto epi_word = [&](int64_t mp, const f32x4 (&ac)[2][4], int e) {
    const int rb = e >> 3, cb = (e >> 1) & 3, d = e & 1;
    const float b0 = bias[cb][2 * d], b1 = bias[cb][2 * d + 1];
    const uint32_t w = pack2(ac[rb][cb][2 * d] + b0, ac[rb][cb][2 * d + 1] + b1);
    ow[cb][d] = w;
    asm volatile("" : "+v"(ow[cb][d]));   // (else sunk to the row block's stores: a VALU burst)
    if constexpr (STATS) {
      float d0 = __uint_as_float(w << 16) - b0, d1 = __uint_as_float(w & 0xffff0000u) - b1;
      if constexpr (TAIL) {   // (a select, no branch in the k-loop)
        const bool ok = mp + rb * 16 + l15 < a.M;
        d0 = ok ? d0 : 0.f;
        d1 = ok ? d1 : 0.f;
      }
      st[0][cb][2 * d] += d0;
      st[1][cb][2 * d] = fmaf(d0, d0, st[1][cb][2 * d]);
      st[0][cb][2 * d + 1] += d1;
      st[1][cb][2 * d + 1] = fmaf(d1, d1, st[1][cb][2 * d + 1]);
      // pinned here: left alone, the compiler sinks every piece's statistics
      // into one VALU burst at the loop latch, outside the MFMA stream
      asm volatile("" : "+v"(st[0][cb][2 * d]), "+v"(st[0][cb][2 * d + 1]), "+v"(st[1][cb][2 * d]),
                   "+v"(st[1][cb][2 * d + 1]));
    }
  };
  // store offsets: lane part (row l15 of the block, its 8 columns; columns
  // past N at an out-of-range offset) into a descriptor that starts at the
  // tile's first row and ends at row M (rows past M are dropped: no masks);
  // soffset 0 (see the file header: an SGPR soffset hides the store-data
  // hazard from the compiler)
  int svo[2][2];
#pragma unroll
  for (int pr = 0; pr < 2; ++pr)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int n = nst + 32 * pr;
      svo[pr][rb] = n < a.N ? (int)(((int64_t)(rb * 16 + l15) * a.ldc + n) * 2) : OOR;
    }
  auto epi_store = [&](int64_t mp, int rb) {
    const __amdgpu_buffer_rsrc_t ct = buf_rsrc(reinterpret_cast<const bf16*>(a.C) + mp * a.ldc,
                                               (a.M - mp) * a.ldc * 2);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      auto s0 = __builtin_amdgcn_permlane16_swap(ow[2 * pr][0], ow[2 * pr + 1][0], false, false);
      auto s1 = __builtin_amdgcn_permlane16_swap(ow[2 * pr][1], ow[2 * pr + 1][1], false, false);
      const u32x4 sv = {s0[0], s1[0], s0[1], s1[1]};
      __builtin_amdgcn_raw_buffer_store_b128(sv, ct, svo[pr][rb], 0, 0);
    }
  };

  // fragments of k-step s sit in xf[s % 4], read two k-steps ahead (16 % 4
  // == 0: the next tile's steps 0 and 1 continue the ring)
  f32x4 accA[2][4], accB[2][4];
  bf16x8 xf[4][2];
  if (ntl > 0) {
    const char* x0b = lds + rowoff;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      xf[kt][0] = xrd(x0b, kt, 0);
      xf[kt][1] = xrd(x0b, kt, 1);
    }
  }
  // tile i: MFMAs into cur, epilogue of tile i-1 (prv) beside them, the DMA
  // of tile i+2 in its first 8 k-steps
  auto body = [&](auto prev_c, int i, f32x4 (&cur)[2][4], const f32x4 (&prv)[2][4]) {
    constexpr bool PREV = decltype(prev_c)::value;
    const char* xb = lds + (i & (WP_NB - 1)) * WP_TILE + rowoff;
    const char* xn = lds + ((i + 1) & (WP_NB - 1)) * WP_TILE + rowoff;
    const int64_t mp = (group + (int64_t)(i - 1) * groups) * WP_TM;
    const TileDma td = tile_dma(i + 2);
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) cur[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < WP_KT; ++kt) {
      if (kt < WP_DPW) piece(td, kt);
      if (kt == WP_KT - 4) {
        // tile i+1 landed (every wave's pieces) and every wave is past tile
        // i-1 (whose buffer tile i+3 refills).  Younger than tile i+1's DMAs:
        // this k-loop's 8 pieces and its first row block's 2 stores
        if constexpr (PREV)
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(WP_DPW + 2) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(WP_DPW) : "memory");
      }
      // ... and tile i+1 is first read one barrier later (from the reads of
      // k-step 14 on): cdna_hip_programming.md, "Read a staged buffer one
      // phase AFTER the wait that retires it"
      if (kt == WP_KT - 2) asm volatile("s_barrier" ::: "memory");
      if (kt + 2 < WP_KT) {
        xf[(kt + 2) & 3][0] = xrd(xb, kt + 2, 0);
        xf[(kt + 2) & 3][1] = xrd(xb, kt + 2, 1);
      } else if (i + 1 < ntl) {   // the next tile's steps 0 and 1
        xf[(kt + 2) & 3][0] = xrd(xn, kt + 2 - WP_KT, 0);
        xf[(kt + 2) & 3][1] = xrd(xn, kt + 2 - WP_KT, 1);
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          cur[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][kt], xf[kt & 3][rb], cur[rb][cb], 0, 0, 0);
      if constexpr (PREV) {
        epi_word(mp, prv, kt);
        if (kt == 7 || kt == 15) epi_store(mp, kt >> 3);
      }
#pragma unroll
      for (int mm = 0; mm < 8; ++mm) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);          // an MFMA
        if (PREV) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // ... then epilogue VALU
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the previous tile's accumulators stay allocated to the end of the tile:
    // left free as the epilogue consumes them, their registers become the
    // destinations of this tile's MFMAs (accumulators moving between
    // registers every k-step) and the epilogue's temporaries alias in-flight
    // MFMA operands -- measured 67 vs 42 us per call without the epilogue
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) asm volatile("" ::"v"(prv[rb][cb]));
  };
  auto finish = [&](int i, const f32x4 (&ac)[2][4]) {   // the last tile's epilogue, alone
    const int64_t mp = (group + (int64_t)i * groups) * WP_TM;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      epi_word(mp, ac, e);
      if (e == 7 || e == 15) epi_store(mp, e >> 3);
    }
  };
  using F = std::integral_constant<bool, false>;
  using T = std::integral_constant<bool, true>;
  if (ntl > 0) {
    body(F{}, 0, accA, accB);
    int i = 1;
    for (; i + 1 < ntl; i += 2) {
      body(T{}, i, accB, accA);
      body(T{}, i + 1, accA, accB);
    }
    if (i < ntl) {
      body(T{}, i, accB, accA);
      finish(i, accB);
    } else {
      finish(i - 1, accA);
    }
  }
  if constexpr (STATS) {
    // per column pair block: 16-lane butterfly, lane (q, m) ends with
    // k = bit2(m), cb = bit3(m), column element r = 2 bit0(m) + bit1(m)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      float x[16];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int r = 0; r < 4; ++r) x[k * 8 + cb * 4 + r] = st[k][2 * pr + cb][r];
      bfly<8, 0x141>(x, (lane & 4) != 0);   // partner lane^7, keep by bit 2
      bfly<4, 0x128>(x, (lane & 8) != 0);   // lane^8, bit 3
      bfly<2, 0xB1>(x, (lane & 1) != 0);    // lane^1, bit 0
      bfly<1, 0x4E>(x, (lane & 2) != 0);    // lane^2, bit 1
      const int k = (lane >> 2) & 1, cb = (lane >> 3) & 1, r = 2 * (lane & 1) + ((lane >> 1) & 1);
      const int n = nw + 32 * pr + cb * 16 + q * 4 + r;
      if (n < a.N) a.part[((int64_t)group * 2 + k) * a.N + n] = x[0];
    }
  }
  // the LDS-DMAs of the two tiles past the last (zeros into buffers this
  // block never reads again) may still be landing: the workgroup's LDS must
  // not be handed to the next workgroup on this CU -- of this launch, or of a
  // kernel running beside it on another stream -- before they have
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool STATS>
dcnr_status launch_wsp(NtArgs a, hipStream_t s, int* nparts) {
  const void* kt = a.M % WP_TM ? (const void*)gemm_wsp_kernel<STATS, true>
                               : (const void*)gemm_wsp_kernel<STATS, false>;
  TRY_ST(set_max_dyn_lds(kt, WP_LDS));
  a.nslices = (int)cdiv(a.N, WP_TN);
  // 32-bit buffer offsets: launch in M-chunks of < 2^29 bytes per operand
  const int64_t maxld = std::max<int64_t>(a.ldx, a.ldc);
  const int64_t mchunk = std::max<int64_t>(WP_TM, ((int64_t(1) << 29) / (maxld * 2)) / WP_TM * WP_TM);
  if (a.M > mchunk) {
    int total = 0;
    for (int64_t m0 = 0; m0 < a.M; m0 += mchunk) {
      NtArgs b = a;
      b.M = std::min(mchunk, a.M - m0);
      b.X = a.X + m0 * a.ldx;
      b.C = (char*)a.C + m0 * a.ldc * 2;
      if (a.part) b.part = a.part + (int64_t)total * 2 * a.N;
      int np = 0;
      TRY_ST(launch_wsp<STATS>(b, s, &np));
      total += np;
    }
    if (nparts) *nparts = total;
    return DCNR_OK;
  }
  a.mtiles = cdiv(a.M, WP_TM);
  const int unit = 8 * a.nslices;
  int grid = std::max(unit, (256 / unit) * unit);
  const int64_t need = a.mtiles * a.nslices;
  if (need < grid) grid = (int)(cdiv(need, unit) * unit);
  a.groups = grid / a.nslices;
  if (nparts) *nparts = a.groups;
  void* args[] = {&a};
  DCNR_HIP(hipLaunchKernel(kt, dim3(grid), dim3(WP_NT), args, WP_LDS, s));
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace

bool gemm_wsp_supported(int epi, int64_t K, int64_t N) {
  return (epi == NT_EPI_BIAS || epi == NT_EPI_BIAS_STATS) && K > 256 && K <= 512 && K % 8 == 0 &&
         N % 8 == 0;
}

dcnr_status gemm_wsp(int epi, const NtArgs& a, hipStream_t s, int* nparts) {
  if (nparts) *nparts = 0;
  if (a.M <= 0 || a.N <= 0) return DCNR_OK;
  if (!gemm_wsp_supported(epi, a.K, a.N) || a.ldx % 8 || a.ldw % 8 || a.ldc % 8 ||
      (epi == NT_EPI_BIAS_STATS && !a.part)) {
    set_error("gemm_wsp: unsupported K=%d N=%d", a.K, a.N);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  return epi == NT_EPI_BIAS_STATS ? launch_wsp<true>(a, s, nparts) : launch_wsp<false>(a, s, nparts);
}

}  // namespace dcnr
