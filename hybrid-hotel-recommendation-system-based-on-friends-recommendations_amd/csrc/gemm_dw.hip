// Weight-gradient GEMM of the bf16 deep tower (gfx950):
//
//   dW[n][k] = sum_b dY[b][n] * X[b][k]      (train.py:225, backward of nn.Linear)
//
// Both operands are batch-major ([B][ld] row-major, the layout the forward
// and the dX GEMM produce), so the contraction runs over their slow index.
// Design (cdna_hip_programming.md, 256^2 tile at ~1 block/CU):
//  * 256(n) x 256(k) output tile per block, 8 waves as 2(n) x 4(k), each wave
//    128 x 64 (8 x 4 MFMA 16x16x32 tiles, 128 fp32 accumulators per lane);
//  * the batch is split S ways (S % 8 == 0); every block of one split runs on
//    one XCD so the split's rows of dY and X come from HBM once;
//  * LDS-DMA staging (buffer_load ... lds, 16 B per lane, no VGPRs), BK = 32
//    batch rows per stage, a ring of 4 stages (32 KiB each) with 3 in flight
//    (counted vmcnt, raw s_barrier: the DMAs stay in flight across it), so
//    ~3 stages of MFMA work cover the HBM latency;
//  * the LDS image is batch-major, rows of 512 B; fragments are read with
//    ds_read_b64_tr_b16 (transposing 4 x 16 blocks).  The 32-B chunks of a
//    row are XOR-swizzled by (row & 7), applied on the per-lane SOURCE
//    address (the DMA destination is lane-linear), so a transposed read's 4
//    rows hit different banks (a 16-row read touches each bank twice: the floor);
//  * out-of-range rows/columns are fetched at an out-of-range buffer offset
//    and read as 0 (branch-free tails);
//  * fp32 split partials go to a TRANSPOSED slab [S][K][ldc] (16-B stores of
//    4 consecutive n; summed and transposed back by splitk_reduce_t).
#include "dcnr_internal.h"

namespace dcnr {
namespace {

// (256 x 128 tiles -- half the split count and so half the fp32 slab, at
// 1.5x the L2->LDS operand bytes and 0.625 instead of 0.375 fragment reads
// per MFMA -- measured +0.5 % per step, profiles/lab/r03at_dw_tiles_ab.txt)
constexpr int BKW = 32, NSTAGE = 4;

// Square T x T output tiles: T = 256 with 8 waves as 2(n) x 4(k) (wave tile
// 128 x 64), T = 128 with 4 waves as 2 x 2 (wave tile 64 x 64).  Smaller tiles
// mean fewer batch splits for the same workgroup count, so a smaller fp32
// slab (S x N x K x 4 bytes written, then read by splitk_reduce_t).
template <int T>
struct DwCfg {
  static constexpr int NW = T == 256 ? 8 : 4;   // waves per workgroup
  static constexpr int WK = NW / 2;              // waves across k (2 across n)
  static constexpr int WTN = T / 2, WTK = T / WK;
  static constexpr int MI = WTN / 16, NJ = WTK / 16;   // 16 x 16 MFMA blocks per wave
  static constexpr int ROWB = T * 2;             // bytes per LDS row (T bf16)
  static constexpr int OPB = BKW * ROWB;         // one operand per stage
  static constexpr int STAGEB = 2 * OPB;         // A + B per stage
  static constexpr int LDS = NSTAGE * STAGEB;    // ring of 4 stages
  static constexpr int RPI = 1024 / ROWB;        // rows per 1-KiB DMA instruction
  static constexpr int IPW = BKW / RPI / NW;     // DMA instructions per operand per wave per stage
  static constexpr int DMAW = 2 * IPW;           // DMA instructions per wave per stage
  static_assert(IPW * RPI * NW == BKW && ROWB / 32 >= 8, "dw tile geometry");
};

// the shipped tile and workgroup target (gemm_dw_splits): 256 x 256 tiles,
// 256 workgroups = 64 splits per 512 x 512 call.  Round 6, with the BN row
// passes folded into the dX GEMMs: 48 splits (a 48 MB slab, -0.29 GB per
// step) ran level with 64 in the step but 92 instead of 79 us alone; 32
// splits +0.8 %.  T = 128 (16 splits: a 16 MB slab, -0.92 GB per step)
// measured 102 us alone against 79 and +8 % per step; with 8 splits (128
// workgroups) 181 us and +22 % (profiles/lab/r06_dw_slab_lab.txt)
constexpr int DW_T = 256, DW_WGS = 256;
// the tail combine's slab loads: default policy (nontemporal measured in
// profiles/lab/r06_xbn_lab.txt)
constexpr bool DW_TAIL_NT = false;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// physical byte offset of logical (row, byte x) inside one operand image
// with RB bytes per row
template <int RB>
__device__ __forceinline__ int swz(int row, int x) {
  return row * RB + ((((x >> 5) ^ (row & 7)) << 5) | (x & 31));
}

// One stage: rows kb..kb+31 of A (cols n0..n0+T-1) and B (cols c0..c0+T-1).
// Each wave-instruction fills 1 KiB = RPI rows; IPW per wave per operand.
template <int T>
__device__ __forceinline__ void stage_load(u32x4 ar, u32x4 br, int64_t lda, int64_t ldb,
                                           int64_t kb, int64_t kend, int n0, int N, int c0, int K,
                                           char* lds_stage, int wave, int lane) {
  using C = DwCfg<T>;
  constexpr int LPR = C::ROWB / 16;            // lanes per row
  const int rsub = lane / LPR, p = lane % LPR;  // row in the group, 16-B position in the row
#pragma unroll
  for (int i = 0; i < C::IPW; ++i) {
    const int row = (wave * C::IPW + i) * C::RPI + rsub;   // 0..31
    const int chunk = ((p >> 1) ^ (row & 7)) * 2 + (p & 1);   // logical 16-B chunk here
    const int64_t b = kb + row;
    const int na = n0 + chunk * 8, ka = c0 + chunk * 8;
    const bool okr = b < kend;
    const int offa = (okr && na < N) ? (int)((b * lda + na) * 2) : OOR;
    const uint32_t dsta = lds_addr(lds_stage) + (wave * C::IPW + i) * 1024;
    dma16(ar, offa, dsta);
    const int offb = (okr && ka < K) ? (int)((b * ldb + ka) * 2) : OOR;
    dma16(br, offb, dsta + C::OPB);
  }
}

// A-operand fragment (16 columns starting at cb, batch rows kk..kk+31):
// lane l gets X[kk + 8*(l>>4) + j][cb + (l&15)], j = 0..7, from the
// batch-major image via two transposed 4x16 block reads.
template <int RB>
__device__ __forceinline__ bf16x8 frag_t(const char* img, int cb, int kk, int lane) {
  const int rk = kk + 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int x = (cb + 4 * (lane & 3)) * 2;
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + swz<RB>(rk, x)));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + swz<RB>(rk + 4, x)));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, c);
}

template <int T>
__global__ __launch_bounds__(DwCfg<T>::NW * 64, 1) void gemm_dw_kernel(DwArgs g) {
  using C = DwCfg<T>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tiles = g.tiles_n * g.tiles_k;
  const int bid = blockIdx.x;
  const int split = (bid % 8) + 8 * (bid / (8 * tiles));
  const int t = (bid / 8) % tiles;
  const int n0 = (t / g.tiles_k) * T, c0 = (t % g.tiles_k) * T;
  const int64_t kbeg = (int64_t)split * g.k_per_split;
  const int64_t kend = min(g.Btot, kbeg + g.k_per_split);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave / C::WK, wk = wave % C::WK;    // wave tile: n wn*WTN.., k wk*WTK..

  const u32x4 ar = rsrc_words(g.A, g.Btot * g.lda * 2);
  const u32x4 br = rsrc_words(g.B, g.Btot * g.ldb * 2);

  f32x4 acc[C::MI][C::NJ];
#pragma unroll
  for (int i = 0; i < C::MI; ++i)
#pragma unroll
    for (int j = 0; j < C::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = kend > kbeg ? (int)((kend - kbeg + BKW - 1) / BKW) : 0;
#pragma unroll
  for (int p = 0; p < NSTAGE - 1; ++p)
    if (p < nst)
      stage_load<T>(ar, br, g.lda, g.ldb, kbeg + (int64_t)p * BKW, kend, n0, g.N, c0, g.K,
                    lds + p * C::STAGEB, wave, lane);
  for (int st = 0; st < nst; ++st) {
    // this wave's DMAs of stage st are done (the younger stages stay in
    // flight), then the barrier makes every wave's part visible and retires
    // stage st-1's reads, so its buffer can be refilled with stage st+3
    if (st + 2 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C::DMAW) : "memory");
    else if (st + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::DMAW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NSTAGE - 1 < nst)
      stage_load<T>(ar, br, g.lda, g.ldb, kbeg + (int64_t)(st + NSTAGE - 1) * BKW, kend, n0, g.N,
                    c0, g.K, lds + ((st + NSTAGE - 1) % NSTAGE) * C::STAGEB, wave, lane);
    const char* ai = lds + (st % NSTAGE) * C::STAGEB;
    const char* bi = ai + C::OPB;
    bf16x8 af[C::MI], bf[C::NJ];
#pragma unroll
    for (int i = 0; i < C::MI; ++i) af[i] = frag_t<C::ROWB>(ai, wn * C::WTN + i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < C::NJ; ++j) bf[j] = frag_t<C::ROWB>(bi, wk * C::WTK + j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < C::MI; ++i)
#pragma unroll
      for (int j = 0; j < C::NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
  }

  // epilogue: acc[i][j][r] = dW[n0 + wn*WTN + i*16 + (lane>>4)*4 + r][c0 + wk*WTK + j*16 + (lane&15)],
  // four consecutive n per lane: the slab is stored transposed ([k][n], row
  // ldc) so each (i, j) is ONE 16-B store (instead of four 4-B stores: the
  // store-issue tail of this kernel); splitk_reduce_t transposes back
  float* out = g.C + (int64_t)split * g.slab_stride;
  const __amdgpu_buffer_rsrc_t cr = buf_rsrc(out, (int64_t)g.K * g.ldc * 4);
#pragma unroll
  for (int i = 0; i < C::MI; ++i)
#pragma unroll
    for (int j = 0; j < C::NJ; ++j) {
      const int k = c0 + wk * C::WTK + j * 16 + (lane & 15);
      const int n = n0 + wn * C::WTN + i * 16 + (lane >> 4) * 4;   // N % 8 == 0: all 4 or none
      const bool ok = n < g.N && k < g.K;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), cr,
                                               ok ? (k * g.ldc + n) * 4 : OOR, 0, 0);
    }

  // the previous call's split-K combine (its slab is complete: that launch
  // ended before this one began on the stream), splitk_reduce_t's tiles
  // dealt over the workgroups, two at a time (256 threads each): a separate
  // launch of it on the side stream waited for CUs beside the dX GEMMs
  if (g.rslab) {
    constexpr int NT = C::NW * 64;
    static_assert(NT == 512, "tail: two 256-thread tile groups");
    __syncthreads();   // every wave is past its last read of the LDS ring
    float(*tt)[RT_N + 1] = reinterpret_cast<float(*)[RT_N + 1]>(lds) + (threadIdx.x / 256) * RT_K;
    // the two halves take tiles (bx, 2j) and (bx, 2j+1): the two 64-B halves
    // of each 128-B slab line, read together (dealt singly, each line came
    // from HBM twice: 134 instead of 67 MB per call by PMC)
    const int nbx = (g.rK + RT_K - 1) / RT_K, nby = (g.rN + RT_N - 1) / RT_N;
    const int npairs = nbx * ((nby + 1) / 2), h = threadIdx.x / 256, idx = threadIdx.x % 256;
    for (int pr = blockIdx.x; pr < npairs; pr += gridDim.x) {
      const int bx = pr % nbx, by = 2 * (pr / nbx) + h;
      if (by < nby) splitk_t_sum<DW_TAIL_NT>(g.rslab, g.rsplits, g.rstride, g.rld, g.rN, g.rK, bx, by, idx, tt);
      __syncthreads();
      if (by < nby) splitk_t_store(g.rN, g.rK, g.rout, g.racc & 1, g.racc >> 1, bx, by, idx, tt);
      __syncthreads();
    }
  }
}

}  // namespace

bool gemm_dw_supported(int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t Btot) {
  return N % 8 == 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         Btot * lda * 2 < (int64_t(1) << 31) && Btot * ldb * 2 < (int64_t(1) << 31);
}

// splits: DW_WGS workgroups per launch, one per CU (32 / 40 / 48 splits
// measured slower or level, profiles/lab/r03z_dw_splits_ab.txt and DW_WGS)
int gemm_dw_splits(int64_t N, int64_t K, int64_t Btot) {
  const int64_t tiles = cdiv(N, DW_T) * cdiv(K, DW_T);
  int64_t s = std::max<int64_t>(8, (DW_WGS / tiles) / 8 * 8);
  while (s > 8 && cdiv(Btot, s) < 2 * BKW) s -= 8;   // at least two stages per split
  return (int)s;
}

dcnr_status gemm_dw(const DwArgs& a0, hipStream_t s) {
  DwArgs a = a0;
  if (!gemm_dw_supported(a.N, a.K, a.lda, a.ldb, a.Btot) || a.splits % 8 || a.splits < 8) {
    set_error("gemm_dw: unsupported N=%d K=%d splits=%d", a.N, a.K, a.splits);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  using C = DwCfg<DW_T>;
  TRY_ST(set_max_dyn_lds((const void*)gemm_dw_kernel<DW_T>, C::LDS));
  a.tiles_n = (int)cdiv(a.N, DW_T);
  a.tiles_k = (int)cdiv(a.K, DW_T);
  const int grid = a.tiles_n * a.tiles_k * a.splits;
  hipLaunchKernelGGL(gemm_dw_kernel<DW_T>, dim3(grid), dim3(C::NW * 64), C::LDS, s, a);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

}  // namespace dcnr
