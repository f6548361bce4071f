// Streaming ceiling, second probe (C3 size, 100M rows, 1000-row segments): is the
// tick's pattern (three read columns + one write column, one 256-thread workgroup
// per segment) limited by the number of concurrent column streams, by the bytes in
// flight per lane, or by the read/write mix?  Variants:
//   seg          the tick's shape (as tools/ubench5.hip), separate output column
//   seg-ro       the same loads, no per-row store (read ceiling of 20 B/row)
//   seg16        16-B loads: each lane loads two adjacent rows per column
//   tile64       columns interleaved per 64-row tile (wants[64] has[64] subs[64]:
//                1280 B contiguous per tile), separate output column
//   tile64-ip    tiled, gets written over the tile's has slots
//   seg512x2     two segments per 512-thread workgroup
//   copy16       16-B copy of one 8-B column (read 0.8 GB, write 0.8 GB)
//   read16       16-B read of the tiled array (2.0 GB)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench6 tools/ubench6.hip
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

constexpr int SEG = 1000;

__global__ __launch_bounds__(256) void k_seg(const double* w, const double* h, const int* s, double* g, int nseg) {
  if ((int)blockIdx.x >= nseg) return;
  const long long lo = (long long)blockIdx.x * SEG;
  double a[4], b[4];
  int c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    const int u = i < SEG ? i : SEG - 1;
    a[k] = w[lo + u];
    b[k] = h[lo + u];
    c[k] = s[lo + u];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    if (i < SEG) __builtin_nontemporal_store(a[k] * 0.5 + b[k] + (double)c[k], g + lo + i);
  }
}

__global__ __launch_bounds__(256) void k_seg_ro(const double* w, const double* h, const int* s, double* g, int nseg) {
  if ((int)blockIdx.x >= nseg) return;
  const long long lo = (long long)blockIdx.x * SEG;
  double a[4], b[4];
  int c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    const int u = i < SEG ? i : SEG - 1;
    a[k] = w[lo + u];
    b[k] = h[lo + u];
    c[k] = s[lo + u];
  }
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc += a[k] * 0.5 + b[k] + (double)c[k];
  if (acc == 12345.678) g[blockIdx.x] = acc;  // never true: keeps the loads
}

// 16-B loads: 500 row pairs per segment, 2 pairs per lane (segments are 1000 rows,
// so every segment starts 8000 B aligned: pairs never straddle)
__global__ __launch_bounds__(256) void k_seg16(const double* w, const double* h, const int* s, double* g, int nseg) {
  if ((int)blockIdx.x >= nseg) return;
  const long long lo = (long long)blockIdx.x * SEG;
  const double2* w2 = (const double2*)(w + lo);
  const double2* h2 = (const double2*)(h + lo);
  const int2* s2 = (const int2*)(s + lo);
  double2 a[2], b[2];
  int2 c[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = k * 256 + threadIdx.x;
    const int u = p < SEG / 2 ? p : SEG / 2 - 1;
    a[k] = w2[u];
    b[k] = h2[u];
    c[k] = s2[u];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = k * 256 + threadIdx.x;
    if (p < SEG / 2) {
      __builtin_nontemporal_store(a[k].x * 0.5 + b[k].x + (double)c[k].x, g + lo + 2 * p);
      __builtin_nontemporal_store(a[k].y * 0.5 + b[k].y + (double)c[k].y, g + lo + 2 * p + 1);
    }
  }
}

// tiled: tile t holds wants at t*160 + [0,64), has at t*160 + [64,128) (8-B units),
// subclients as 64 ints at t*160 + 128 .. +160.  Row r -> tile r>>6, lane r&63.
__device__ __forceinline__ long long tw(long long r) { return (r >> 6) * 160 + (r & 63); }
template <bool IP>
__global__ __launch_bounds__(256) void k_tile(double* t, double* g, int nseg) {
  if ((int)blockIdx.x >= nseg) return;
  const long long lo = (long long)blockIdx.x * SEG;
  double a[4], b[4];
  int c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    const long long r = lo + (i < SEG ? i : SEG - 1);
    const long long o = tw(r);
    a[k] = t[o];
    b[k] = t[o + 64];
    c[k] = ((const int*)(t + (r >> 6) * 160 + 128))[r & 63];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + threadIdx.x;
    if (i < SEG) {
      const double v = a[k] * 0.5 + b[k] + (double)c[k];
      if (IP)
        __builtin_nontemporal_store(v, t + tw(lo + i) + 64);
      else
        __builtin_nontemporal_store(v, g + lo + i);
    }
  }
}

__global__ __launch_bounds__(512) void k_seg2(const double* w, const double* h, const int* s, double* g, int nseg) {
  const int seg = blockIdx.x * 2 + (threadIdx.x >> 8);
  if (seg >= nseg) return;
  const long long lo = (long long)seg * SEG;
  const int t = threadIdx.x & 255;
  double a[4], b[4];
  int c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + t;
    const int u = i < SEG ? i : SEG - 1;
    a[k] = w[lo + u];
    b[k] = h[lo + u];
    c[k] = s[lo + u];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = k * 256 + t;
    if (i < SEG) __builtin_nontemporal_store(a[k] * 0.5 + b[k] + (double)c[k], g + lo + i);
  }
}

__global__ __launch_bounds__(256) void k_copy16(const double2* src, double2* dst, long long n2) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const double2 v = src[i];
    __builtin_nontemporal_store(v.x, &dst[i].x);
    __builtin_nontemporal_store(v.y, &dst[i].y);
  }
}

__global__ __launch_bounds__(256) void k_read16(const double2* src, double* out, long long n2) {
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const double2 v = src[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 100000000LL;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  double *w, *h, *g, *t;
  int* s;
  CK(hipMalloc(&w, n * 8));
  CK(hipMalloc(&h, n * 8));
  CK(hipMalloc(&g, n * 8));
  CK(hipMalloc(&s, n * 4));
  CK(hipMalloc(&t, (n / 64 + 1) * 1280));
  CK(hipMemset(w, 0, n * 8));
  CK(hipMemset(h, 0, n * 8));
  CK(hipMemset(g, 0, n * 8));
  CK(hipMemset(s, 0, n * 4));
  CK(hipMemset(t, 0, (n / 64 + 1) * 1280));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("%-28s %8.1f us  %6.2f TB/s (%.0f B/row)\n", name, us, bytes / us / 1e6, bytes / (double)n);
  };
  const int nseg = (int)(n / SEG);
  for (int rep = 0; rep < 2; ++rep) {
    run("seg", 28.0 * n, [&] { k_seg<<<nseg, 256>>>(w, h, s, g, nseg); });
    run("seg-ro", 20.0 * n, [&] { k_seg_ro<<<nseg, 256>>>(w, h, s, g, nseg); });
    run("seg16", 28.0 * n, [&] { k_seg16<<<nseg, 256>>>(w, h, s, g, nseg); });
    run("tile64", 28.0 * n, [&] { k_tile<false><<<nseg, 256>>>(t, g, nseg); });
    run("tile64-ip", 28.0 * n, [&] { k_tile<true><<<nseg, 256>>>(t, g, nseg); });
    run("seg512x2", 28.0 * n, [&] { k_seg2<<<(nseg + 1) / 2, 512>>>(w, h, s, g, nseg); });
    // copy/read of the same byte volume as the tick (2.8 GB)
    run("copy16 (w -> g)", 16.0 * n, [&] { k_copy16<<<cus * 16, 256>>>((const double2*)w, (double2*)g, n / 2); });
    run("read16", 20.0 * n, [&] { k_read16<<<cus * 16, 256>>>((const double2*)t, g, (20LL * n) / 16 < (n / 64) * 80 ? (20LL * n) / 16 : (n / 64) * 80); });
  }
  return 0;
}
