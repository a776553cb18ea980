// Cross-wave RAW of LDS-DMA under a co-resident LDS-heavy kernel (gfx950 lab,
// "DMA -> counted vmcnt -> barrier -> another wave's read,
// beside an LDS-heavy co-resident kernel").
//
// Kernel P (probe) has gemm_wsp's shape: 4 waves, a 4-buffer ring of 32-KB
// tiles (128 KB of LDS), each wave filling 8 of a tile's 32 rows by LDS-DMA
// (1-KB pieces from a 1 GiB table, random rows: HBM misses).  Per step t:
// issue tile t+1 (8 pieces per wave), `s_waitcnt vmcnt(8)` (tile t's pieces
// are the older ones), `s_barrier`, then EVERY wave reads all 32 rows of tile
// t and compares them with the table; one more barrier before the next step
// (tile t's buffer is refilled at step t+3).  Younger operations at the wait:
//   mode 0: tile t+1's real DMAs (the steady state),
//   mode 1: 8 empty-descriptor DMAs (num_records 0) instead -- tile t+1 is
//           loaded one step later, after the read (gemm_wsp's last tiles),
//   mode 2: as 0 plus two 16-B stores after the DMAs, vmcnt(10).
// Kernel B runs beside it on another stream: one 32-KB workgroup per CU,
// ds_write / ds_read of its own pattern in a loop (lds_iso.hip's B), with few
// registers so its waves share P's SIMDs.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lab_bin/lds_dma_raw tools/lab/lds_dma_raw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void dma16s(u32x4 rsrc, int voff, int soff, uint32_t lds_dst) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, %3 offen lds"
      :
      : "v"(voff), "s"(rsrc), "{m0}"(lds_dst), "s"(soff)
      : "memory");
}
__device__ __forceinline__ u32x4 rsrc(const void* p, unsigned bytes) {
  const uint64_t a = (uint64_t)p;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xFFFFu, bytes, 0x00020000u};
}
__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}

constexpr int TILE = 32768, NB = 4, ROWS = 32;

// table row of tile row r at step t (uniform per block)
__device__ __forceinline__ unsigned trow(unsigned seed, int t, int r, unsigned rows) {
  return mix(seed ^ (blockIdx.x * 0x9E3779B1u) ^ ((unsigned)t * 0x7FEB352Du) ^ ((unsigned)r * 0x846CA68Bu)) % rows;
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void probe(const unsigned* big, unsigned rows, unsigned* sink, int steps,
                                                unsigned seed, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t base = lds_addr(lds);
  const u32x4 rb = rsrc(big, 0xFFFFFFFFu), rz = rsrc(big, 0u), rs = rsrc(sink, 1u << 20);
  auto issue = [&](int t, bool zero) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const int r = wave * 8 + d;
      const unsigned row = __builtin_amdgcn_readfirstlane(trow(seed, t, r, rows));
      dma16s(zero ? rz : rb, lane * 16, (int)(row * 1024u),
             __builtin_amdgcn_readfirstlane(base + (t % NB) * TILE + r * 1024));
    }
  };
  unsigned bad = 0, zeros = 0;
  issue(0, false);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < steps; ++t) {
    if constexpr (MODE == 1) {
      issue(t + 1, true);          // zeros into tile t+1's buffer (reloaded below)
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    } else if constexpr (MODE == 0) {
      issue(t + 1, false);
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    } else {
      issue(t + 1, false);
      asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\tbuffer_store_dwordx4 %0, %1, %2, 0 offen offset:1024"
                   ::"v"(u32x4{1u, 2u, 3u, 4u}), "v"((int)((blockIdx.x * 4 + wave) * 2048 % (1 << 20)) + lane * 16 % 1024),
                   "s"(rs)
                   : "memory");
      asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
    }
    // every wave reads every row of tile t
    const char* tb = lds + (t % NB) * TILE;
#pragma unroll 4
    for (int r = 0; r < ROWS; ++r) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(tb + r * 1024 + lane * 16);
      const unsigned w0 = trow(seed, t, r, rows) * 256u + lane * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bad += v[j] != w0 + j;
        zeros += v[j] == 0u && w0 + j != 0u;
      }
    }
    if constexpr (MODE == 1) {
      // the real tile t+1 now: the zeros are in, every wave has read tile t
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue(t + 1, false);
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  atomicAdd(&out[0], bad);
  atomicAdd(&out[1], zeros);
}

// B: its own pattern through 32 KB of LDS, over and over
__global__ __launch_bounds__(256) void lds_hog(int rounds, unsigned tag, unsigned* bad) {
  extern __shared__ __attribute__((aligned(16))) unsigned lb[];
  const unsigned seed = tag ^ (blockIdx.x * 0x9E3779B9u);
  unsigned nbad = 0;
  for (int r = 0; r < rounds; ++r) {
    for (int i = threadIdx.x; i < 8192; i += 256) lb[i] = seed ^ i ^ r;
    __syncthreads();
    for (int i = threadIdx.x; i < 8192; i += 256) nbad += lb[(i * 33) & 8191] != (seed ^ ((i * 33) & 8191) ^ r);
    __syncthreads();
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned rows = 1u << 20;   // 1 GiB
  unsigned *big, *sink, *out;
  CK(hipMalloc(&big, (size_t)rows * 1024));
  CK(hipMalloc(&sink, 1u << 20));
  CK(hipMalloc(&out, 16));
  {
    const size_t n = (size_t)rows * 256;
    unsigned* h = (unsigned*)malloc(n * 4);
    for (size_t i = 0; i < n; ++i) h[i] = (unsigned)i;
    CK(hipMemcpy(big, h, n * 4, hipMemcpyHostToDevice));
    free(h);
  }
  const void* k[3] = {(const void*)probe<0>, (const void*)probe<1>, (const void*)probe<2>};
  const char* name[3] = {"younger = next tile's real DMAs, vmcnt(8)", "younger = 8 empty-descriptor DMAs, vmcnt(8)",
                         "younger = next tile's DMAs + 2 stores, vmcnt(10)"};
  CK(hipFuncSetAttribute((const void*)lds_hog, hipFuncAttributeMaxDynamicSharedMemorySize, 32768));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int steps = 400;
  for (int hog = 0; hog < 2; ++hog)
    for (int m = 0; m < 3; ++m) {
      CK(hipFuncSetAttribute(k[m], hipFuncAttributeMaxDynamicSharedMemorySize, NB * TILE));
      unsigned tot[3] = {0, 0, 0};
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemset(out, 0, 16));
        if (hog) hipLaunchKernelGGL(lds_hog, dim3(cus), dim3(256), 32768, s2, 3000, 0xabcdu + rep, out + 2);
        unsigned seed = 0x5151u + rep * 131u + m;
        int st = steps;
        void* args[] = {&big, (void*)&rows, &sink, &st, &seed, &out};
        CK(hipLaunchKernel(k[m], dim3(cus), dim3(256), args, NB * TILE, s1));
        CK(hipDeviceSynchronize());
        unsigned h[3];
        CK(hipMemcpy(h, out, 12, hipMemcpyDeviceToHost));
        for (int j = 0; j < 3; ++j) tot[j] += h[j];
      }
      const double words = 5.0 * cus * 4 * steps * ROWS * 64 * 4;
      printf("%s mode %d (%s): wrong %u (zeros %u) of %.0f words read; hog errors %u\n",
             hog ? "beside lds_hog" : "alone        ", m, name[m], tot[0], tot[1], words, tot[2]);
    }
  return 0;
}
