// Kernel lab for gemm_dw_kernel: rebuilds csrc/gemm_dw.hip with DW_LAB_MODE
// (1: no MFMA, 2: no stage loads, 4: no epilogue stores) and times it alone.
#include "../hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc/gemm_dw.hip"

#include <cstdarg>
#include <cstdio>
#include <cstring>
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

int main() {
  const int64_t B = 131072;
  const int N = 512, K = 512;
  dcnr::bf16 *A, *X;
  float* slab;
  const int S = dcnr::gemm_dw_splits(N, K, B);
  (void)hipMalloc(&A, B * N * 2); (void)hipMalloc(&X, B * K * 2);
  (void)hipMalloc(&slab, (size_t)S * N * K * 4);
  {   // random bf16 in [-1, 1) (constant data runs at a higher clock than real data)
    std::vector<uint16_t> h(B * (size_t)std::max(N, K));
    uint32_t st = 12345;
    for (auto& v : h) {
      st = st * 1664525u + 1013904223u;
      const float f = (float)(st >> 8) / 8388608.f - 1.f;
      v = (uint16_t)(__builtin_bit_cast(uint32_t, f) >> 16);
    }
    (void)hipMemcpy(A, h.data(), B * N * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(X, h.data() + 3, B * K * 2, hipMemcpyHostToDevice);
  }
  dcnr::DwArgs a;
  std::memset(&a, 0, sizeof(a));
  a.A = A; a.lda = N; a.B = X; a.ldb = K; a.C = slab; a.ldc = K; a.slab_stride = (int64_t)N * K;
  a.Btot = B; a.k_per_split = (B + S - 1) / S; a.N = N; a.K = K; a.splits = S;
  for (int i = 0; i < 3; ++i) dcnr::gemm_dw(a, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < 20; ++i) dcnr::gemm_dw(a, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("dw mode %d  S=%d  %.1f us  %.0f TF/s  %s\n", DW_LAB_MODE, S, ms * 1e3 / 20,
         2.0 * B * N * K / (ms * 1e3 / 20) / 1e6, hipGetErrorString(hipGetLastError()));
  return 0;
}
