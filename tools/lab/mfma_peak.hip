// Sustained dense bf16 MFMA rate of this box, registers only (no memory in the
// loop): every wave issues independent v_mfma_f32_16x16x32_bf16 (or
// 32x32x16) on operands loaded once from random data (all-zero operands
// draw less power and clock higher than real tiles).  The ceiling the
// production kernels' "fraction of the nominal 2.5 PF/s" is read against.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form -o tools/lab_bin/mfma_peak tools/lab/mfma_peak.hip
// (without the flag the compiler shuffles the 16x16 accumulators through
// ~50 AGPR moves per 8 MFMAs: a broken measurement)
//   tools/lab_bin/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// 8 independent 16x16x32 accumulators per wave: 8 MFMAs in flight covers the
// dependent-issue latency
__global__ __launch_bounds__(256) void mfma16_kernel(const bf16x8* __restrict__ src, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[2];
  for (int i = 0; i < 4; ++i) a[i] = src[(blockIdx.x * 8 + i) * 64 + lane];
  for (int i = 0; i < 2; ++i) b[i] = src[(blockIdx.x * 8 + 4 + i) * 64 + lane];
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 3], b[i >> 2], acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 4 independent 32x32x16 accumulators per wave
__global__ __launch_bounds__(256) void mfma32_kernel(const bf16x8* __restrict__ src, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[2], b[2];
  for (int i = 0; i < 2; ++i) a[i] = src[(blockIdx.x * 8 + i) * 64 + lane];
  for (int i = 0; i < 2; ++i) b[i] = src[(blockIdx.x * 8 + 2 + i) * 64 + lane];
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i & 1], b[i >> 1], acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) s += acc[i][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int maxblocks = cus * 8;
  std::vector<uint16_t> h((size_t)maxblocks * 8 * 64 * 8);
  srand(1);
  for (auto& x : h) x = (uint16_t)(0x3c00 + (rand() & 0x7ff)) ^ (uint16_t)((rand() & 1) << 15);  // +-[1, 4)
  bf16x8* src;
  float* out;
  CK(hipMalloc(&src, h.size() * 2));
  CK(hipMalloc(&out, (size_t)maxblocks * 256 * 4));
  CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20000;
  for (int shape = 0; shape < 2; ++shape) {
    for (int wps = 1; wps <= 2; ++wps) {   // waves per SIMD: blocks of 4 waves per CU
      const int blocks = cus * wps;
      auto launch = [&]() {
        if (shape == 0) hipLaunchKernelGGL(mfma16_kernel, dim3(blocks), dim3(256), 0, 0, src, out, iters);
        else hipLaunchKernelGGL(mfma32_kernel, dim3(blocks), dim3(256), 0, 0, src, out, iters);
      };
      launch();
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      // flops per MFMA: 16x16x32x2 = 16384 (8 per iteration), 32x32x16x2 = 32768 (4 per iteration)
      const double fl = (double)blocks * 4 * iters * (shape == 0 ? 8.0 * 16384 : 4.0 * 32768);
      printf("%s  %d wave(s)/SIMD  %.3f ms  %.1f TF/s  (%.3f of 2.5 PF/s)\n",
             shape == 0 ? "mfma_f32_16x16x32_bf16" : "mfma_f32_32x32x16_bf16", wps, best, fl / best / 1e9,
             fl / best / 1e9 / 2500.0);
    }
  }
  CK(hipFree(src));
  CK(hipFree(out));
  return 0;
}
