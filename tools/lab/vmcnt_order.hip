// Counted-vmcnt retirement order of LDS-DMA (gfx950 lab).
//
// Question: does `s_waitcnt vmcnt(N)` still cover an OLDER LDS-DMA when the N
// younger vector-memory operations are
//   mode 0: LDS-DMAs through an empty descriptor (num_records = 0: every lane
//           out of range -- gemm_wsp's "past-the-end zero tiles"),
//   mode 1: real LDS-DMAs of L2-hot lines (control),
//   mode 2: buffer stores of L2-hot lines (control: gemm_wsp's C stores),
//   mode 3: gemm_wsp's exact mix before the last tile's wait: 8 empty-descriptor
//           DMAs + 2 stores, vmcnt(10)?
// Per iteration each wave writes a sentinel into its own 1-KB LDS slot, issues
// ONE LDS-DMA of a cold 1-KB line (a random row of a 1 GiB buffer, so it misses
// to HBM) into that slot, then the N younger operations, then vmcnt(N), then
// reads the slot back itself (the issuing wave: no barrier involved).  A slot
// that still holds the sentinel means the wait retired before the older DMA
// had landed: the counted wait is not an in-order wait for that mix.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lab_bin/vmcnt_order tools/lab/vmcnt_order.hip
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
// the library's dma16 (csrc/dcnr_internal.h)
__device__ __forceinline__ void dma16(u32x4 rsrc, int off, uint32_t lds_dst) {
  asm volatile(
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %1, 0 offen lds"
      :
      : "v"(off), "s"(rsrc), "{m0}"(lds_dst)
      : "memory");
}
__device__ __forceinline__ void st4(u32x4 rsrc, int off, unsigned v) {
  asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(v), "v"(off), "s"(rsrc) : "memory");
}
__device__ __forceinline__ u32x4 rsrc(const void* p, unsigned bytes) {
  const uint64_t a = (uint64_t)p;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xFFFFu, bytes, 0x00020000u};
}
__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}

constexpr unsigned SENT = 0xFFFFFFFFu;

// big: word i = i over `rows` 1-KB rows; hot: 16 KB, L2-resident after the first touch
template <int MODE>
__global__ __launch_bounds__(256, 1) void probe(const unsigned* big, unsigned rows, unsigned* hot, int iters,
                                                unsigned seed, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  char* slot = lds + wave * 1024;
  const uint32_t slot_a = __builtin_amdgcn_readfirstlane(lds_addr(slot));
  const uint32_t young_a = __builtin_amdgcn_readfirstlane(lds_addr(lds + 4096 + wave * 8192));
  const u32x4 rb = rsrc(big, 0xFFFFFFFFu);
  const u32x4 rz = rsrc(big, 0u);            // empty descriptor: every lane out of range
  const u32x4 rh = rsrc(hot, 16384u);
  unsigned stale = 0, wrong = 0;
  for (int it = 0; it < iters; ++it) {
    *reinterpret_cast<u32x4*>(slot + lane * 16) = u32x4{SENT, SENT, SENT, SENT};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned row = __builtin_amdgcn_readfirstlane(
        mix(seed ^ (blockIdx.x * 0x9E3779B1u) ^ (wave * 0x7FEB352Du) ^ (it * 0x846CA68Bu)) % rows);
    dma16(rb, (int)(row * 1024u + lane * 16), slot_a);                      // the OLD operation
    if constexpr (MODE == 0) {
#pragma unroll
      for (int d = 0; d < 8; ++d) dma16(rz, lane * 16, young_a + d * 1024);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int d = 0; d < 8; ++d) dma16(rh, d * 1024 + lane * 16, young_a + d * 1024);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int d = 0; d < 8; ++d) st4(rh, (wave * 8 + d) * 256 + lane * 4, it);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
#pragma unroll
      for (int d = 0; d < 8; ++d) dma16(rz, lane * 16, young_a + d * 1024);
#pragma unroll
      for (int d = 0; d < 2; ++d) st4(rh, (wave * 8 + d) * 256 + lane * 4, it);
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    }
    const u32x4 v = *reinterpret_cast<const u32x4*>(slot + lane * 16);
    const unsigned w0 = row * 256u + lane * 4;
    for (int j = 0; j < 4; ++j) {
      stale += v[j] == SENT;
      wrong += v[j] != SENT && v[j] != w0 + j;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  atomicAdd(&out[0], stale);
  atomicAdd(&out[1], wrong);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned rows = 1u << 20;   // 1 GiB
  unsigned *big, *hot, *out;
  CK(hipMalloc(&big, (size_t)rows * 1024));
  CK(hipMalloc(&hot, 16384));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(hot, 0, 16384));
  {
    const size_t n = (size_t)rows * 256;
    unsigned* h = (unsigned*)malloc(n * 4);
    for (size_t i = 0; i < n; ++i) h[i] = (unsigned)i;
    CK(hipMemcpy(big, h, n * 4, hipMemcpyHostToDevice));
    free(h);
  }
  const void* k[4] = {(const void*)probe<0>, (const void*)probe<1>, (const void*)probe<2>, (const void*)probe<3>};
  const char* name[4] = {"8 empty-descriptor LDS-DMAs, vmcnt(8)", "8 L2-hot LDS-DMAs, vmcnt(8)",
                         "8 L2-hot buffer stores, vmcnt(8)", "8 empty-descriptor LDS-DMAs + 2 stores, vmcnt(10)"};
  const int iters = 200, grid = cus * 2;
  for (int m = 0; m < 4; ++m) {
    CK(hipFuncSetAttribute(k[m], hipFuncAttributeMaxDynamicSharedMemorySize, 4096 + 4 * 8192));
    unsigned tot[2] = {0, 0};
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipMemset(out, 0, 8));
      unsigned seed = 0x1234u + rep * 77u + m;
      int it = iters;
      void* args[] = {&big, (void*)&rows, &hot, &it, &seed, &out};
      CK(hipLaunchKernel(k[m], dim3(grid), dim3(256), args, 4096 + 4 * 8192, 0));
      CK(hipDeviceSynchronize());
      unsigned h[2];
      CK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
      tot[0] += h[0];
      tot[1] += h[1];
    }
    const double words = 5.0 * grid * 4 * iters * 64 * 4;
    printf("mode %d (%s): stale %u, wrong %u of %.0f words (%.4f stale)\n", m, name[m], tot[0], tot[1], words,
           tot[0] / words);
  }
  return 0;
}
