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
}  // namespace dcnr

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atol(argv[1]) : 131072;
  const int K = argc > 2 ? atoi(argv[2]) : 512, N = argc > 3 ? atoi(argv[3]) : 512;
  dcnr::bf16 *X, *W, *C;
  float* b;
  hipMalloc(&X, M * K * 2); hipMalloc(&W, (size_t)N * K * 2); hipMalloc(&C, M * N * 2);
  hipMalloc(&b, N * 4);
  hipMemset(X, 0x3c, M * K * 2); hipMemset(W, 0x3c, (size_t)N * K * 2); hipMemset(b, 0, N * 4);
  dcnr::NtArgs a;
  std::memset(&a, 0, sizeof(a));
  a.X = X; a.ldx = K; a.M = M; a.K = K; a.W = W; a.ldw = K; a.N = N; a.C = C; a.ldc = N; a.bias = b;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) dcnr::gemm_nt(dcnr::NT_EPI_BIAS, a, 0);
  const int it = 20;
  hipEventRecord(e0, 0);
  for (int i = 0; i < it; ++i) dcnr::gemm_nt(dcnr::NT_EPI_BIAS, a, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double us = ms * 1e3 / it;
  printf("mode %d  M=%ld K=%d N=%d  %.1f us  %.0f TF/s  %.2f TB/s\n", NT_LAB_MODE, (long)M, K, N, us,
         2.0 * M * N * K / us / 1e6, (M * K * 2.0 + M * N * 2.0) / us / 1e6);
  return 0;
}
