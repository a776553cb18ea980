// LDS isolation between workgroups of two kernels sharing CUs (gfx950 lab):
// kernel A (128 KB dynamic LDS, one block per CU) fills its LDS -- by ds_write
// or by LDS-DMA (buffer_load ... lds, M0 = its own LDS address) -- and
// re-checks it while kernel B (32 KB, many blocks, another stream) does the
// same with its own pattern.  Counts words that changed under either.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lab_bin/lds_iso tools/lab/lds_iso.hip
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

// 16 B per lane from `off` of the buffer into LDS lds_dst + 16 * lane
__device__ __forceinline__ void dma16(u32x4 rsrc, int off, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(rsrc), "s"(lds_dst)
      : "memory");
}

// words: LDS bytes / 4; pattern word i of block b = tag ^ (b * 0x9E3779B9u) ^ i
template <bool DMA>
__global__ __launch_bounds__(256) void fill_check(const unsigned* src, int words, unsigned tag, int rounds,
                                                  unsigned* bad) {
  extern __shared__ __attribute__((aligned(16))) unsigned lds[];
  const unsigned seed = tag ^ (blockIdx.x * 0x9E3779B9u);
  if constexpr (DMA) {
    // src holds the pattern of seed 0: word i = i; the DMA copies it and the
    // check below xors the seed in software
    const u32x4 rs = {(unsigned)(uintptr_t)src, (unsigned)((uintptr_t)src >> 32) & 0xFFFFu,
                      (unsigned)(words * 4), 0x00020000u};
    const uint32_t base = lds_addr(lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int p = w; p < words / 256; p += 4)   // 1 KB pieces
      dma16(rs, p * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(base + p * 1024));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    for (int i = threadIdx.x; i < words; i += 256) lds[i] = seed ^ i;
    __syncthreads();
  }
  unsigned nbad = 0;
  for (int r = 0; r < rounds; ++r) {
    for (int i = threadIdx.x; i < words; i += 256) {
      const unsigned want = DMA ? (unsigned)i : (seed ^ i);
      if (lds[i] != want) ++nbad;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int wa = 128 * 1024 / 4, wb = 32 * 1024 / 4;
  unsigned *src, *bad;
  CK(hipMalloc(&src, wa * 4));
  CK(hipMalloc(&bad, 8));
  unsigned* h = (unsigned*)malloc(wa * 4);
  for (int i = 0; i < wa; ++i) h[i] = i;
  CK(hipMemcpy(src, h, wa * 4, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)fill_check<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  CK(hipFuncSetAttribute((const void*)fill_check<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (int mode = 0; mode < 2; ++mode) {
    unsigned tot[2] = {0, 0};
    for (int rep = 0; rep < 20; ++rep) {
      CK(hipMemset(bad, 0, 8));
      // A: 128 KB per block, one per CU (B launched right after, on another stream)
      if (mode)
        hipLaunchKernelGGL(fill_check<true>, dim3(cus), dim3(256), 128 * 1024, s1, src, wa, 0x1234u + rep, 200, bad);
      else
        hipLaunchKernelGGL(fill_check<false>, dim3(cus), dim3(256), 128 * 1024, s1, src, wa, 0x1234u + rep, 200, bad);
      hipLaunchKernelGGL(fill_check<false>, dim3(cus * 8), dim3(256), 32 * 1024, s2, src, wb, 0xabcdu + rep, 50,
                         bad + 1);
      CK(hipDeviceSynchronize());
      unsigned hb[2];
      CK(hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost));
      tot[0] += hb[0];
      tot[1] += hb[1];
    }
    printf("A filled by %s: words changed under A %u, under B %u (20 runs)\n", mode ? "LDS-DMA" : "ds_write",
           tot[0], tot[1]);
  }
  return 0;
}
