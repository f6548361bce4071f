// Streaming ceiling for the follower-layout writeback tick's access pattern (C3
// size, 100M rows): read wants f64, has f64, subclients i32; write gets f64 (28 B
// per row), into a separate column or in place over has.  Flat kernels with no
// reductions, 8-B and 16-B lanes: the rate no tick kernel of this pattern can beat.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench5 tools/ubench5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t err_ = (x);                                                          \
    if (err_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__global__ __launch_bounds__(256) void k_flat8(const double* w, const double* h, const int* s, double* g,
                                               long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double v = w[i] * 0.5 + h[i] + (double)s[i];
    __builtin_nontemporal_store(v, g + i);
  }
}

__global__ __launch_bounds__(256) void k_flat16(const double2* w, const double2* h, const int2* s, double2* g,
                                                long long n2) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const double2 a = w[i], b = h[i];
    const int2 c = s[i];
    __builtin_nontemporal_store(a.x * 0.5 + b.x + (double)c.x, &g[i].x);
    __builtin_nontemporal_store(a.y * 0.5 + b.y + (double)c.y, &g[i].y);
  }
}

// one 256-thread workgroup per 1000-row segment, 4 rows per lane, all loads first
// (the tick kernel's shape without its reductions)
__global__ __launch_bounds__(256) void k_seg(const double* w, const double* h, const int* s, double* g, int nseg) {
  const long long lo = (long long)blockIdx.x * 1000;
  if ((int)blockIdx.x >= nseg) return;
  double a[4], b[4];
  int c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    const int u = i < 1000 ? i : 999;
    a[k] = w[lo + u];
    b[k] = h[lo + u];
    c[k] = s[lo + u];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    if (i < 1000) __builtin_nontemporal_store(a[k] * 0.5 + b[k] + (double)c[k], g + lo + i);
  }
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 100000000LL;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  double *w, *h, *g;
  int* s;
  CK(hipMalloc(&w, n * 8));
  CK(hipMalloc(&h, n * 8));
  CK(hipMalloc(&g, n * 8));
  CK(hipMalloc(&s, n * 4));
  CK(hipMemset(w, 0, n * 8));
  CK(hipMemset(h, 0, n * 8));
  CK(hipMemset(g, 0, n * 8));
  CK(hipMemset(s, 0, n * 4));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = 28.0 * (double)n;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("%-34s %8.1f us  %6.2f TB/s (28 B/row)\n", name, us, bytes / us / 1e6);
  };
  for (int wpc : {8, 16, 32}) {
    const int grid = cus * wpc;
    char nm[64];
    snprintf(nm, sizeof nm, "flat8 separate, %d WG/CU", wpc);
    run(nm, [&] { k_flat8<<<grid, 256>>>(w, h, s, g, n); });
    snprintf(nm, sizeof nm, "flat8 in place, %d WG/CU", wpc);
    run(nm, [&] { k_flat8<<<grid, 256>>>(w, h, s, h, n); });
    snprintf(nm, sizeof nm, "flat16 separate, %d WG/CU", wpc);
    run(nm, [&] { k_flat16<<<grid, 256>>>((const double2*)w, (const double2*)h, (const int2*)s, (double2*)g, n / 2); });
  }
  const int nseg = (int)(n / 1000);
  run("seg 1000 rows/WG separate", [&] { k_seg<<<nseg, 256>>>(w, h, s, g, nseg); });
  run("seg 1000 rows/WG in place", [&] { k_seg<<<nseg, 256>>>(w, h, s, h, nseg); });
  return 0;
}
