// Streaming ceiling for the writeback tick's exact access pattern (C3 size):
// read wants f64, has f64, subclients i32, expiry i64; write has f64 + expiry i64
// in place (44 B per row).  Compares 8-B vs 16-B lanes, flat grid-stride vs one
// workgroup per 1000-row segment with block reductions between load and store.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench4 tools/ubench4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t err_ = (x);                                                          \
    if (err_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

struct Cols {
  double* w;
  double* h;
  int* s;
  long long* e;
};

__global__ __launch_bounds__(256) void k_flat8(Cols c, long long n, long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double w = c.w[i], h = c.h[i];
    const int s = c.s[i];
    const long long e = c.e[i];
    __builtin_nontemporal_store((now > e) ? 0.0 : w * 0.5 + h + (double)s, c.h + i);
    __builtin_nontemporal_store(now + s, c.e + i);
  }
}

__global__ __launch_bounds__(256) void k_flat16(Cols c, long long n2, long long now) {
  const double2* w2 = (const double2*)c.w;
  double2* h2 = (double2*)c.h;
  const int2* s2 = (const int2*)c.s;
  longlong2* e2 = (longlong2*)c.e;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const double2 w = w2[i], h = h2[i];
    const int2 s = s2[i];
    const longlong2 e = e2[i];
    double2 g;
    g.x = (now > e.x) ? 0.0 : w.x * 0.5 + h.x + (double)s.x;
    g.y = (now > e.y) ? 0.0 : w.y * 0.5 + h.y + (double)s.y;
    longlong2 x;
    x.x = now + s.x;
    x.y = now + s.y;
    __builtin_nontemporal_store(g.x, &h2[i].x);
    __builtin_nontemporal_store(g.y, &h2[i].y);
    __builtin_nontemporal_store(x.x, &e2[i].x);
    __builtin_nontemporal_store(x.y, &e2[i].y);
  }
}

__device__ __forceinline__ double block_sum(double v, double* lds) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = lds[0] + lds[1] + lds[2] + lds[3];
  __syncthreads();
  return r;
}

// one 256-thread workgroup per S-row segment, R rows per lane (8-B lanes)
template <int R, int BATCH, int NRED>
__global__ __launch_bounds__(256) void k_seg8(Cols c, int S, long long now) {
  __shared__ double lds[4];
  const long long lo = (long long)blockIdx.x * S;
  const int t = threadIdx.x;
  double w[R], h[R];
  int s[R];
  long long e[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = k * 256 + t;
    const unsigned u = (unsigned)(i < S ? i : S - 1);
    w[k] = c.w[lo + u];
    h[k] = c.h[lo + u];
    s[k] = c.s[lo + u];
    e[k] = c.e[lo + u];
    if (BATCH < R && (k + 1) % BATCH == 0 && k + 1 < R) __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < R; ++k)
    if (k * 256 + t < S && !(now > e[k])) acc += w[k] + (double)s[k];
  double tot = 0.0;
  for (int r = 0; r < NRED; ++r) tot += block_sum(acc + tot, lds);
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = k * 256 + t;
    if (i >= S) continue;
    __builtin_nontemporal_store((now > e[k]) ? 0.0 : w[k] * 0.5 + h[k] + tot, c.h + lo + i);
    __builtin_nontemporal_store(now + s[k], c.e + lo + i);
  }
}

// same with 16-B lanes: lane t owns rows 2*(k*256+t) and +1 of the pair-aligned range
template <int P, int NRED>
__global__ __launch_bounds__(256) void k_seg16(Cols c, int S, long long now) {
  __shared__ double lds[4];
  const long long lo = (long long)blockIdx.x * S;
  const long long alo = lo & ~1LL;
  const int pre = (int)(lo - alo);
  const int n2 = (S + pre + 1) >> 1;
  const int t = threadIdx.x;
  double2 w[P], h[P];
  int2 s[P];
  longlong2 e[P];
  const double2* w2 = (const double2*)(c.w + alo);
  const double2* h2 = (const double2*)(c.h + alo);
  const int2* s2 = (const int2*)(c.s + alo);
  const longlong2* e2 = (const longlong2*)(c.e + alo);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int i = k * 256 + t;
    const unsigned u = (unsigned)(i < n2 ? i : n2 - 1);
    w[k] = w2[u];
    h[k] = h2[u];
    s[k] = s2[u];
    e[k] = e2[u];
  }
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int r0 = 2 * (k * 256 + t) - pre;
    if (r0 >= 0 && r0 < S && !(now > e[k].x)) acc += w[k].x + (double)s[k].x;
    if (r0 + 1 < S && !(now > e[k].y)) acc += w[k].y + (double)s[k].y;
  }
  double tot = 0.0;
  for (int r = 0; r < NRED; ++r) tot += block_sum(acc + tot, lds);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int r0 = 2 * (k * 256 + t) - pre;
    const double g0 = (now > e[k].x) ? 0.0 : w[k].x * 0.5 + h[k].x + tot;
    const double g1 = (now > e[k].y) ? 0.0 : w[k].y * 0.5 + h[k].y + tot;
    double* hp = c.h + lo + r0;
    long long* ep = c.e + lo + r0;
    if (r0 >= 0 && r0 + 1 < S) {
      typedef double vd2 __attribute__((ext_vector_type(2)));
      typedef long long vl2 __attribute__((ext_vector_type(2)));
      vd2 g = {g0, g1};
      vl2 x = {now + s[k].x, now + s[k].y};
      __builtin_nontemporal_store(g, (vd2*)hp);
      __builtin_nontemporal_store(x, (vl2*)ep);
    } else {
      if (r0 >= 0 && r0 < S) {
        __builtin_nontemporal_store(g0, hp);
        __builtin_nontemporal_store(now + s[k].x, ep);
      }
      if (r0 + 1 >= 0 && r0 + 1 < S) {
        __builtin_nontemporal_store(g1, hp + 1);
        __builtin_nontemporal_store(now + s[k].y, ep + 1);
      }
    }
  }
}

// reference points: float4 copy, read-only sum of the four columns, out-of-place outputs,
// plain (temporal) stores
__global__ __launch_bounds__(256) void k_copy16(const double2* __restrict__ a, double2* __restrict__ b, long long n2) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void k_read8(Cols c, long long n, long long now, double* out) {
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long e = c.e[i];
    acc += (now > e) ? 0.0 : c.w[i] * 0.5 + c.h[i] + (double)c.s[i];
  }
  if (acc == 12345.0) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_flat8_oop(Cols c, double* __restrict__ g, long long* __restrict__ x, long long n,
                                                   long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double w = c.w[i], h = c.h[i];
    const int s = c.s[i];
    const long long e = c.e[i];
    __builtin_nontemporal_store((now > e) ? 0.0 : w * 0.5 + h + (double)s, g + i);
    __builtin_nontemporal_store(now + s, x + i);
  }
}
__global__ __launch_bounds__(256) void k_flat8_plain(Cols c, long long n, long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double w = c.w[i], h = c.h[i];
    const int s = c.s[i];
    const long long e = c.e[i];
    c.h[i] = (now > e) ? 0.0 : w * 0.5 + h + (double)s;
    c.e[i] = now + s;
  }
}
// write-only: the two output columns
__global__ __launch_bounds__(256) void k_write8(Cols c, long long n, long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    __builtin_nontemporal_store((double)i, c.h + i);
    __builtin_nontemporal_store(now + i, c.e + i);
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / reps;
}

int main(int argc, char** argv) {
  const long long N = argc > 1 ? atoll(argv[1]) : 100000000LL;
  const int S = argc > 2 ? atoi(argv[2]) : 1000;
  const int reps = 20;
  Cols c;
  CK(hipMalloc((void**)&c.w, (N + 2) * 8));
  CK(hipMalloc((void**)&c.h, (N + 2) * 8));
  CK(hipMalloc((void**)&c.s, (N + 2) * 4));
  CK(hipMalloc((void**)&c.e, (N + 2) * 8));
  std::vector<double> hw(N);
  for (long long i = 0; i < N; ++i) hw[i] = (double)(i % 997) * 0.001;
  CK(hipMemcpy(c.w, hw.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(c.h, hw.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset((void*)c.s, 0, N * 4));
  CK(hipMemset((void*)c.e, 0x7f, N * 8));
  const double bytes = 44.0 * N;
  const long long now = 1;
  auto report = [&](const char* name, float ms) {
    printf("%-28s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  {
    double *A, *B, *G;
    long long* X;
    CK(hipMalloc((void**)&A, N * 16));
    CK(hipMalloc((void**)&B, N * 16));
    CK(hipMemset(A, 0, N * 16));
    const double cb = 32.0 * N;
    for (int grid : {2048, 8192}) {
      float ms = time_it([&] { k_copy16<<<grid, 256>>>((const double2*)A, (double2*)B, N); }, reps);
      printf("copy16 %dB grid=%d %8.1f us  %7.1f GB/s\n", (int)(cb / 1e6), grid, ms * 1e3, cb / (ms * 1e-3) / 1e9);
    }
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipMalloc((void**)&G, N * 8));
    CK(hipMalloc((void**)&X, N * 8));
    for (int grid : {2048, 8192}) {
      float ms = time_it([&] { k_read8<<<grid, 256>>>(c, N, now, G); }, reps);
      printf("read8 (28 B/row) grid=%d %8.1f us  %7.1f GB/s\n", grid, ms * 1e3, 28.0 * N / (ms * 1e-3) / 1e9);
      ms = time_it([&] { k_write8<<<grid, 256>>>(c, N, now); }, reps);
      printf("write8 (16 B/row) grid=%d %8.1f us  %7.1f GB/s\n", grid, ms * 1e3, 16.0 * N / (ms * 1e-3) / 1e9);
      char nm[64];
      snprintf(nm, sizeof nm, "flat8 oop grid=%d", grid);
      report(nm, time_it([&] { k_flat8_oop<<<grid, 256>>>(c, G, X, N, now); }, reps));
      snprintf(nm, sizeof nm, "flat8 plain grid=%d", grid);
      report(nm, time_it([&] { k_flat8_plain<<<grid, 256>>>(c, N, now); }, reps));
    }
    CK(hipFree(G));
    CK(hipFree(X));
  }
  if (argc > 3) return 0;
  for (int grid : {2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "flat8 grid=%d", grid);
    report(nm, time_it([&] { k_flat8<<<grid, 256>>>(c, N, now); }, reps));
    snprintf(nm, sizeof nm, "flat16 grid=%d", grid);
    report(nm, time_it([&] { k_flat16<<<grid, 256>>>(c, N / 2, now); }, reps));
  }
  const int nseg = (int)(N / S);
  for (int pass = 0; pass < 2; ++pass) {
    report("seg8 R4 B4 red0", time_it([&] { k_seg8<4, 4, 0><<<nseg, 256>>>(c, S, now); }, reps));
    report("seg8 R4 B2 red0", time_it([&] { k_seg8<4, 2, 0><<<nseg, 256>>>(c, S, now); }, reps));
    report("seg8 R4 B4 red4", time_it([&] { k_seg8<4, 4, 4><<<nseg, 256>>>(c, S, now); }, reps));
    report("seg8 R4 B2 red4", time_it([&] { k_seg8<4, 2, 4><<<nseg, 256>>>(c, S, now); }, reps));
    report("seg16 P2 red0", time_it([&] { k_seg16<2, 0><<<nseg, 256>>>(c, S, now); }, reps));
    report("seg16 P2 red4", time_it([&] { k_seg16<2, 4><<<nseg, 256>>>(c, S, now); }, reps));
  }
  return 0;
}
