// Host-memory probe for the row reader's slabs: cost of pinning (hipHostMalloc,
// malloc + hipHostRegister, with and without transparent huge pages) and D2H
// throughput into pinned vs pageable memory. Build: hipcc -O2 pin_probe.cpp
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  const size_t n = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 256) << 20;
  void* d = nullptr;
  if (hipMalloc(&d, n) != hipSuccess) return 1;
  (void)hipMemset(d, 1, n);
  (void)hipDeviceSynchronize();
  double t = now();
  void* h1 = nullptr;
  if (hipHostMalloc(&h1, n, hipHostMallocDefault) != hipSuccess) return 2;
  const double t_hm = now() - t;
  t = now();
  void* h1b = nullptr;
  if (hipHostMalloc(&h1b, n, hipHostMallocNonCoherent) != hipSuccess) return 2;
  const double t_hmnc = now() - t;
  // malloc'd, touched, then registered
  t = now();
  void* h2 = aligned_alloc(1 << 21, n);
  memset(h2, 0, n);
  const double t_touch = now() - t;
  t = now();
  const int rr = hipHostRegister(h2, n, hipHostRegisterDefault);
  const double t_reg = now() - t;
  // THP-advised, touched, registered
  void* h3 = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  madvise(h3, n, MADV_HUGEPAGE);
  t = now();
  memset(h3, 0, n);
  const double t_touch_thp = now() - t;
  t = now();
  const int rr3 = hipHostRegister(h3, n, hipHostRegisterDefault);
  const double t_reg_thp = now() - t;
  // pageable target, touched
  void* h4 = malloc(n);
  memset(h4, 0, n);
  auto d2h = [&](void* h) {
    (void)hipMemcpy(h, d, n, hipMemcpyDeviceToHost);
    const double s = now();
    for (int i = 0; i < 3; ++i) (void)hipMemcpy(h, d, n, hipMemcpyDeviceToHost);
    return 3.0 * n / (now() - s) / 1e9;
  };
  printf("{\"MB\": %zu, \"hipHostMalloc_s\": %.4f, \"hipHostMalloc_noncoherent_s\": %.4f, \"malloc_touch_s\": %.4f, "
         "\"hipHostRegister_s\": %.4f, \"reg_rc\": %d, \"thp_touch_s\": %.4f, \"thp_register_s\": %.4f, \"reg3_rc\": %d, "
         "\"d2h_pinned_GBps\": %.1f, \"d2h_pinned_nc_GBps\": %.1f, \"d2h_registered_GBps\": %.1f, \"d2h_registered_thp_GBps\": %.1f, "
         "\"d2h_pageable_GBps\": %.1f}\n",
         n >> 20, t_hm, t_hmnc, t_touch, t_reg, rr, t_touch_thp, t_reg_thp, rr3, d2h(h1), d2h(h1b), d2h(h2), d2h(h3), d2h(h4));
  return 0;
}
