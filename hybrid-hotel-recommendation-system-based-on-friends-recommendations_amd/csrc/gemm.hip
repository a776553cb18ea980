// MFMA GEMMs for the DCN-R deep tower (gfx950).
//
//   C[M,N] = A[M,K] . B[N,K]^T      A/B either k-fastest ("N") or stored
//                                    transposed ("T": m/n fastest)
//
// The deep tower needs three shapes per Linear layer (train.py:143,105,109):
//   forward   h = x W^T + b        A = x [B][K] (N), B = W [H][K] (N)
//   dX        dx = dy W            A = dy [B][H] (N), B = W^T packed [K][H] (N)
//   dW        dW = dy^T x          A = dy (T), B = x (T), contraction over the
//                                  batch, split-K slabs reduced deterministically
//
// bf16 path: v_mfma_f32_16x16x32_bf16, fp32 accumulate.  fp32 (parity) path:
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains).  128x128 block tile, 4 waves
// of 64x64, register-staged double-buffered LDS.  Transposed operands are
// kept in their memory layout in LDS and read with ds_read_b64_tr_b16 (bf16)
// or strided ds_read_b32 (fp32), so no operand is ever transposed in HBM.
// Block ids are remapped so that the tiles sharing an A row-panel run on one
// XCD (blocks b, b+8, ... share an XCD's L2).
#include "dcnr_internal.h"

#include <type_traits>

namespace dcnr {
namespace {

constexpr int BM = 128, BN = 128, NT = 256;

template <typename T> struct Cfg;
template <> struct Cfg<bf16> { static constexpr int BK = 64, KS = 32, V = 8; };
template <> struct Cfg<float> { static constexpr int BK = 16, KS = 4, V = 4; };

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T, bool TR, int ROWS_M>
struct TileLayout {
  static constexpr int BK = Cfg<T>::BK, V = Cfg<T>::V;
  static constexpr int ROWS = TR ? BK : ROWS_M;         // LDS rows
  static constexpr int COLS = (TR ? ROWS_M : BK) + V;   // + 16 B pad
  static constexpr int SIZE = ROWS * COLS;
  static constexpr int CHUNKS = ROWS_M * BK / V / NT;   // 16-B chunks per thread
};

// Load one tile of an operand (logical [rows=m][k]) into registers.
template <typename T, bool TR, int ROWS_M>
__device__ __forceinline__ void load_tile(uint4* r,
                                          const T* __restrict__ P, int64_t ld, int64_t m0,
                                          int64_t mlim, int64_t k0, int64_t klim) {
  using L = TileLayout<T, TR, ROWS_M>;
  constexpr int V = L::V, BK = L::BK;
#pragma unroll
  for (int i = 0; i < L::CHUNKS; ++i) {
    int c = threadIdx.x + i * NT;
    int64_t m, k;
    if (!TR) { m = m0 + c / (BK / V); k = k0 + (c % (BK / V)) * V; }
    else { k = k0 + c / (ROWS_M / V); m = m0 + (c % (ROWS_M / V)) * V; }
    if (m < mlim && k < klim) {
      const T* src = TR ? (P + k * ld + m) : (P + m * ld + k);
      r[i] = *reinterpret_cast<const uint4*>(src);
    } else {
      r[i] = make_uint4(0, 0, 0, 0);
    }
  }
}

template <typename T, bool TR, int ROWS_M>
__device__ __forceinline__ void store_tile(T* lds, const uint4* r) {
  using L = TileLayout<T, TR, ROWS_M>;
  constexpr int V = L::V, BK = L::BK;
#pragma unroll
  for (int i = 0; i < L::CHUNKS; ++i) {
    int c = threadIdx.x + i * NT;
    int row, col;
    if (!TR) { row = c / (BK / V); col = (c % (BK / V)) * V; }
    else { row = c / (ROWS_M / V); col = (c % (ROWS_M / V)) * V; }
    *reinterpret_cast<uint4*>(lds + row * L::COLS + col) = r[i];
  }
}

// bf16 MFMA fragment (16 rows starting at mb within the tile, k-step kk):
// lane l holds X[mb + (l&15)][kk + 8*(l>>4) + j], j = 0..7.
template <bool TR, int COLS>
__device__ __forceinline__ bf16x8 frag_bf16(const bf16* lds, int mb, int kk, int lane) {
  if (!TR) {
    return *reinterpret_cast<const bf16x8*>(lds + (mb + (lane & 15)) * COLS + kk + 8 * (lane >> 4));
  } else {
    // LDS holds [k][m]; two transposed 4x16 block reads give 8 consecutive k.
    int rk = kk + 8 * (lane >> 4) + ((lane & 15) >> 2);
    int cm = mb + 4 * (lane & 3);
    const bf16* p0 = lds + rk * COLS + cm;
    const bf16* p1 = p0 + 4 * COLS;
    s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(bf16x8, c);
  }
}

// f32 MFMA 16x16x4 fragment: lane l holds X[mb + (l&15)][kk + (l>>4)].
template <bool TR, int COLS>
__device__ __forceinline__ float frag_f32(const float* lds, int mb, int kk, int lane) {
  if (!TR) return lds[(mb + (lane & 15)) * COLS + kk + (lane >> 4)];
  return lds[(kk + (lane >> 4)) * COLS + mb + (lane & 15)];
}

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nwg) {
  // bijective: the blocks that share an XCD (bid % 8) get a contiguous range
  int64_t q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <typename T, bool AT, bool BT, int EPI, typename TO>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs g) {
  using LA = TileLayout<T, AT, BM>;
  using LB = TileLayout<T, BT, BN>;
  constexpr int BK = Cfg<T>::BK, KS = Cfg<T>::KS;
  __shared__ __attribute__((aligned(16))) T lds[2 * (LA::SIZE + LB::SIZE)];

  const int64_t ntl = (g.N + BN - 1) / BN;
  int64_t t;
  int split;
  if (g.xcd_split) {
    // split-K over the batch: every output tile of one split runs on one XCD
    // (blocks b, b+8, ... share an L2), so the split's rows of both operands
    // are fetched from HBM once and re-read from L2 by the other tiles
    const int64_t ntiles = ((g.M + BM - 1) / BM) * ntl;
    const int64_t bid = blockIdx.x;
    split = (int)((bid % 8) + 8 * (bid / (8 * ntiles)));
    t = (bid / 8) % ntiles;
  } else {
    t = xcd_remap(blockIdx.x, gridDim.x);
    split = blockIdx.y;
  }
  const int64_t tm = t / ntl, tn = t % ntl;
  const int64_t m0 = tm * BM, n0 = tn * BN;
  const int64_t kbeg = (int64_t)split * g.k_per_split;
  const int64_t kend = min(g.K, kbeg + g.k_per_split);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const T* A = (const T*)g.A;
  const T* B = (const T*)g.B;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[LA::CHUNKS], rb[LB::CHUNKS];
  int ntiles = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;
  if (ntiles > 0) {
    load_tile<T, AT, BM>(ra, A, g.lda, m0, g.M, kbeg, kend);
    load_tile<T, BT, BN>(rb, B, g.ldb, n0, g.N, kbeg, kend);
    store_tile<T, AT, BM>(lds, ra);
    store_tile<T, BT, BN>(lds + LA::SIZE, rb);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ntiles; ++kt) {
    const bool more = kt + 1 < ntiles;
    if (more) {
      int64_t k1 = kbeg + (int64_t)(kt + 1) * BK;
      load_tile<T, AT, BM>(ra, A, g.lda, m0, g.M, k1, kend);
      load_tile<T, BT, BN>(rb, B, g.ldb, n0, g.N, k1, kend);
    }
    const T* a_s = lds + cur * (LA::SIZE + LB::SIZE);
    const T* b_s = a_s + LA::SIZE;
#pragma unroll
    for (int kk = 0; kk < BK; kk += KS) {
      if constexpr (std::is_same<T, bf16>::value) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag_bf16<AT, LA::COLS>(a_s, wm * 64 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag_bf16<BT, LB::COLS>(b_s, wn * 64 + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      } else {
        float af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag_f32<AT, LA::COLS>(a_s, wm * 64 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag_f32<BT, LB::COLS>(b_s, wn * 64 + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      T* nb = lds + (cur ^ 1) * (LA::SIZE + LB::SIZE);
      store_tile<T, AT, BM>(nb, ra);
      store_tile<T, BT, BN>(nb + LA::SIZE, rb);
    }
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: acc[i][j][r] -> C[m0+wm*64+i*16+(lane>>4)*4+r][n0+wn*64+j*16+(lane&15)]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wn * 64 + j * 16 + (lane & 15);
    if (n >= g.N) continue;
    float bias = (EPI != EPI_SPLITK && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= g.M) continue;
        float v = acc[i][j][r];
        if constexpr (EPI == EPI_SPLITK) {
          ((float*)g.C)[(int64_t)split * g.slab_stride + m * g.ldc + n] = v;
        } else {
          v += bias;
          if constexpr (EPI == EPI_STORE_RESID) v += St<T>::ld((const T*)g.resid + m * g.ldr + n);
          St<TO>::st((TO*)g.C + m * g.ldc + n, v);
        }
      }
    }
  }
}

template <typename T, bool AT, bool BT, int EPI, typename TO>
dcnr_status launch(const GemmArgs& a, int splits, hipStream_t s) {
  int64_t mt = cdiv(a.M, BM), ntl = cdiv(a.N, BN);
  GemmArgs b = a;
  dim3 grid((unsigned)(mt * ntl), (unsigned)splits);
  b.xcd_split = 0;
  if (EPI == EPI_SPLITK && splits % 8 == 0) {
    b.xcd_split = 1;
    grid = dim3((unsigned)(mt * ntl * splits), 1);
  }
  hipLaunchKernelGGL((gemm_kernel<T, AT, BT, EPI, TO>), grid, dim3(NT), 0, s, b);
  DCNR_LAUNCH_CHECK();
  return DCNR_OK;
}

template <typename T, int EPI, typename TO>
dcnr_status dispatch_t(bool a_t, bool b_t, const GemmArgs& a, int splits, hipStream_t s) {
  if (!a_t && !b_t) return launch<T, false, false, EPI, TO>(a, splits, s);
  if (a_t && b_t) return launch<T, true, true, EPI, TO>(a, splits, s);
  set_error("gemm: unsupported transpose combination");
  return DCNR_UNSUPPORTED_SHAPE;
}

template <typename T>
dcnr_status dispatch(bool a_t, bool b_t, int epi, const GemmArgs& a, int splits, hipStream_t s) {
  switch (epi) {
    case EPI_STORE:
      return a.out_f32 ? dispatch_t<T, EPI_STORE, float>(a_t, b_t, a, splits, s)
                       : dispatch_t<T, EPI_STORE, T>(a_t, b_t, a, splits, s);
    case EPI_STORE_RESID:
      return dispatch_t<T, EPI_STORE_RESID, T>(a_t, b_t, a, splits, s);
    case EPI_SPLITK:
      return dispatch_t<T, EPI_SPLITK, float>(a_t, b_t, a, splits, s);
  }
  set_error("gemm: bad epilogue %d", epi);
  return DCNR_BAD_ARG;
}

}  // namespace

dcnr_status gemm(int precision, bool a_t, bool b_t, int epi, const GemmArgs& a, int splits,
                 hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return DCNR_OK;
  bool ok = a.lda % 8 == 0 && a.ldb % 8 == 0;
  ok = ok && (a_t ? a.M % 8 == 0 : a.K % 8 == 0);
  ok = ok && (b_t ? a.N % 8 == 0 : a.K % 8 == 0);
  ok = ok && (splits <= 1 || a.k_per_split % Cfg<float>::BK == 0);
  if (!ok) {
    set_error("gemm: unsupported extents M=%lld N=%lld K=%lld lda=%lld ldb=%lld", (long long)a.M,
              (long long)a.N, (long long)a.K, (long long)a.lda, (long long)a.ldb);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  return precision == DCNR_PREC_BF16 ? dispatch<bf16>(a_t, b_t, epi, a, splits, s)
                                     : dispatch<float>(a_t, b_t, epi, a, splits, s);
}

}  // namespace dcnr
