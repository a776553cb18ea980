// Lab: rocPRIM radix_sort_pairs at the embedding-backward size (14 tables x
// B = 131072 (key = global table row, 21 bits; value = sample)), timed alone.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <cstdint>

static void run(const char* name, size_t n, const uint32_t* rows, int T, int B, int bits) {
  std::vector<uint32_t> k(n), v(n);
  uint32_t st = 1;
  std::vector<uint32_t> base(T);
  base[0] = 0;
  for (int t = 1; t < T; ++t) base[t] = base[t - 1] + rows[t - 1];
  for (int t = 0; t < T; ++t)
    for (int b = 0; b < B; ++b) {
      st = st * 1664525u + 1013904223u;
      k[(size_t)t * B + b] = base[t] + (st >> 8) % rows[t];
      v[(size_t)t * B + b] = b;
    }
  uint32_t *ki, *ko, *vi, *vo;
  hipMalloc(&ki, n * 4); hipMalloc(&ko, n * 4); hipMalloc(&vi, n * 4); hipMalloc(&vo, n * 4);
  hipMemcpy(ki, k.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(vi, v.data(), n * 4, hipMemcpyHostToDevice);
  size_t tb = 0;
  rocprim::radix_sort_pairs(nullptr, tb, ki, ko, vi, vo, n, 0, bits);
  void* tmp;
  hipMalloc(&tmp, tb);
  for (int i = 0; i < 3; ++i) rocprim::radix_sort_pairs(tmp, tb, ki, ko, vi, vo, n, 0, bits);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 20; ++i) rocprim::radix_sort_pairs(tmp, tb, ki, ko, vi, vo, n, 0, bits);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint32_t> ks(n), vs(n);
  hipMemcpy(ks.data(), ko, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(vs.data(), vo, n * 4, hipMemcpyDeviceToHost);
  bool ok = true;
  for (size_t i = 1; i < n; ++i)
    if (ks[i] < ks[i - 1] || (ks[i] == ks[i - 1] && vs[i] < vs[i - 1])) { ok = false; break; }
  printf("%-28s n=%zu bits=%d: %.1f us, temp %zu B, stable-sorted %d\n", name, n, bits, ms * 1e3 / 20, tb, ok);
  hipFree(ki); hipFree(ko); hipFree(vi); hipFree(vo); hipFree(tmp);
}

int main() {
  const int B = 131072;
  const uint32_t all[14] = {1000000, 100000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000, 1000};
  run("all 14 tables", (size_t)B * 14, all, 14, B, 21);
  run("user+item", (size_t)B * 2, all, 2, B, 21);
  run("12 cat tables", (size_t)B * 12, all + 2, 12, B, 14);
  run("1 cat table", (size_t)B, all + 2, 1, B, 10);
  return 0;
}
