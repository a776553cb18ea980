// MFMA issue-rate probe (lab, not part of the library): v_mfma_f32_16x16x32_bf16
// back to back on register operands, NACC independent accumulators per wave,
// W waves per workgroup (1 workgroup per CU), an s_barrier every PER MFMAs.
// Prints the MFMA-pipe utilisation implied by the wall time at the measured
// clock: busy = 16 cycles x MFMAs per SIMD / (time x clock).
//   mfma_lab <waves per WG> <mfma per wave> <mfma between barriers>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int NACC>
__global__ void mfma_kernel(int n, int per, float* out) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * (lane + i)); b[i] = (__bf16)(0.002f * (lane - i)); }
  f32x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < n; it += per) {
    for (int k = 0; k < per; k += NACC) {
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    }
    if (per < n) __syncthreads();
  }
  float t = 0.f;
  for (int j = 0; j < NACC; ++j) t += acc[j][0];
  if (t == 1234.5f) out[0] = t;
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 8;
  const int n = argc > 2 ? atoi(argv[2]) : 4096;
  const int per = argc > 3 ? atoi(argv[3]) : 128;
  float* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(mfma_kernel<8>, dim3(256), dim3(64 * waves), 0, 0, n, per, out);
  hipEventRecord(e0);
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(mfma_kernel<8>, dim3(256), dim3(64 * waves), 0, 0, n, per, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it;
  const double per_simd = (double)n * waves / 4;           // MFMAs per SIMD
  printf("waves/WG %d  mfma/wave %d  barrier every %d: %.1f us, %.1f cycles per MFMA per SIMD at 2.4 GHz "
         "(busy %.2f)\n", waves, n, per, us, us * 2400.0 / per_simd, 16.0 * per_simd / (us * 2400.0));
  return 0;
}
