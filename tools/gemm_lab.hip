// Kernel lab for gemm_nt_kernel: rebuilds csrc/gemm_nt.hip with NT_LAB_MODE
// (see there) and times one cfg3-shaped call.  Build + run: tools/gemm_lab.sh
#include "../hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc/gemm_nt.hip"

#include <cstdarg>
#include <cstring>
#include <cstdio>
#include <vector>

namespace dcnr {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fprintf(stderr, "\n");
}
dcnr_status set_max_dyn_lds(const void* k, size_t bytes) {
  return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess
             ? DCNR_OK : DCNR_HIP_ERROR;
}
}  // namespace dcnr

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atol(argv[1]) : 131072;
  const int K = argc > 2 ? atoi(argv[2]) : 512, N = argc > 3 ? atoi(argv[3]) : 512;
  const int ldx = argc > 4 ? atoi(argv[4]) : K, ldc = argc > 5 ? atoi(argv[5]) : N;
  const int epi = argc > 6 ? atoi(argv[6]) : 0;   // dcnr::NtEpi
  dcnr::bf16 *X, *W, *C, *R, *H, *T;
  float *b, *mean, *istd, *part;
  hipMalloc(&X, M * ldx * 2); hipMalloc(&W, (size_t)N * K * 2); hipMalloc(&C, M * ldc * 4);
  hipMalloc(&R, M * ldc * 2); hipMalloc(&H, M * ldc * 2); hipMalloc(&T, M * ldc * 2);
  hipMalloc(&b, N * 4); hipMalloc(&mean, N * 4); hipMalloc(&istd, N * 4);
  hipMalloc(&part, (size_t)8192 * 2 * N * 4);
  hipMemset(mean, 0, N * 4); hipMemset(istd, 0, N * 4);
  {  // random bf16 in [-1, 1): MFMA power (and so clocks) depend on the data
    std::vector<uint16_t> h(std::max<size_t>(M * ldx, (size_t)N * K));
    uint32_t st = 12345;
    for (auto& v : h) {
      st = st * 1664525u + 1013904223u;
      const float f = (float)(st >> 8) / 8388608.f - 1.f;
      v = (uint16_t)(__builtin_bit_cast(uint32_t, f) >> 16);
    }
    hipMemcpy(X, h.data(), M * ldx * 2, hipMemcpyHostToDevice);
    hipMemcpy(W, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice);
    for (auto* p : {R, H, T}) hipMemcpy(p, h.data(), std::min(M * ldx, M * ldc) * 2, hipMemcpyHostToDevice);
    hipMemset(b, 0, N * 4);
  }
  dcnr::NtArgs a;
  std::memset(&a, 0, sizeof(a));
  a.X = X; a.ldx = ldx; a.M = M; a.K = K; a.W = W; a.ldw = K; a.N = N; a.C = C; a.ldc = ldc; a.bias = b;
  a.R = R; a.ldr = ldc; a.H = H; a.ldh = ldc; a.T = T; a.ldt = ldc; a.hscale = 2.5f;
  a.mean = mean; a.invstd = istd; a.part = part;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) dcnr::gemm_nt(epi, a, 0);
  const int it = 20;
  hipEventRecord(e0, 0);
  for (int i = 0; i < it; ++i) dcnr::gemm_nt(epi, a, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double us = ms * 1e3 / it;
  printf("epi %d (%s)  waves %d rb %d depth %d  mode %d  M=%ld K=%d N=%d ldx=%d ldc=%d  %.1f us  %.0f TF/s  %.2f TB/s\n", epi, hipGetErrorString(hipGetLastError()), NT_WAVES, NT_RB, NT_DEPTH, NT_LAB_MODE, (long)M, K, N, ldx, ldc, us,
         2.0 * M * N * K / us / 1e6, (M * K * 2.0 + M * N * 2.0) / us / 1e6);
  return 0;
}
