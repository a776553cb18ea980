// Kernel lab for gather_cross_fwd_kernel: rebuilds csrc/gather_cross.hip with
// GC_LAB_MODE (see there) and times the cfg3 forward gather (B=131072, bf16 x0).
#include "../hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc/gather_cross.hip"

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>

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
  const int64_t B = argc > 1 ? atol(argv[1]) : 131072;
  const int E = 32, K = 12, F = 8, L = 3;
  const int64_t rows[14] = {1000000, 100000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000};
  dcnr::GatherDesc g;
  std::memset(&g, 0, sizeof(g));
  g.n_tab = 2 + K; g.n_num = F;
  int off = 0;
  for (int t = 0; t < g.n_tab; ++t) {
    float* p; (void)hipMalloc(&p, rows[t] * E * 4); (void)hipMemset(p, 0, rows[t] * E * 4);
    g.tab[t] = p; g.rows[t] = rows[t]; g.width[t] = E; g.off[t] = off; off += E;
  }
  g.D = off + F;
  const int D = g.D, ldx = (D + 7) / 8 * 8;
  dcnr::CrossParams cp;
  std::memset(&cp, 0, sizeof(cp));
  cp.L = L;
  float* wts; (void)hipMalloc(&wts, (2 * L + 1) * D * 4); (void)hipMemset(wts, 0, (2 * L + 1) * D * 4);
  for (int l = 0; l < L; ++l) { cp.w[l] = wts + l * D; cp.b[l] = wts + (L + l) * D; }
  cp.wf_cross = wts + 2 * L * D;
  std::vector<int64_t> hu(B), hi(B), hc(B * K);
  std::mt19937_64 rng(0);
  for (int64_t b = 0; b < B; ++b) { hu[b] = rng() % rows[0]; hi[b] = rng() % rows[1]; }
  for (auto& c : hc) c = rng() % 1000;
  int64_t *u, *it, *c; float *num, *zc; dcnr::bf16* x0; int* err;
  (void)hipMalloc(&u, B * 8); (void)hipMalloc(&it, B * 8); (void)hipMalloc(&c, B * K * 8);
  (void)hipMalloc(&num, B * F * 4); (void)hipMalloc(&zc, B * 4); (void)hipMalloc(&x0, B * ldx * 2);
  (void)hipMalloc(&err, 4);
  (void)hipMemcpy(u, hu.data(), B * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(it, hi.data(), B * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(c, hc.data(), B * K * 8, hipMemcpyHostToDevice);
  (void)hipMemset(num, 0, B * F * 4);
  auto run = [&] {
    dcnr::gather_cross_fwd(DCNR_PREC_BF16, g, cp, u, it, c, num, B, x0, ldx, zc, err, 0, 0);
  };
  for (int i = 0; i < 3; ++i) run();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int iters = 20;
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) run();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / iters;
  printf("gather mode %d  B=%ld  %.1f us  %.2f TB/s of 2852 B/sample\n", GC_LAB_MODE, (long)B, us,
         2852.0 * B / us / 1e6);
  (void)hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
