// ubench.hip — access-pattern ceilings for the apportionment tick on MI355X.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench tools/ubench.hip
// Each variant moves the tick's algorithmic bytes (read wants/has/sub/expiry,
// write gets/expiry = 48 B per row) over N rows in segments of S rows.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t err_ = (x);                                                       \
    if (err_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// 1. flat grid-stride stream, 8 B per lane per column
__global__ __launch_bounds__(256) void k_flat8(const double* __restrict__ w, const double* __restrict__ h,
                                              const long long* __restrict__ s, const long long* __restrict__ e,
                                              double* __restrict__ g, long long* __restrict__ x, long long n,
                                              long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double ww = w[i], hh = h[i];
    const long long ss = s[i], ee = e[i];
    g[i] = (now > ee) ? 0.0 : ww * 0.5 + hh + (double)ss;
    x[i] = now + ss;
  }
}

// 2. flat stream, 16 B per lane per column (two rows per lane)
__global__ __launch_bounds__(256) void k_flat16(const double2* __restrict__ w, const double2* __restrict__ h,
                                               const longlong2* __restrict__ s, const longlong2* __restrict__ e,
                                               double2* __restrict__ g, longlong2* __restrict__ x, long long n2,
                                               long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const double2 ww = w[i], hh = h[i];
    const longlong2 ss = s[i], ee = e[i];
    double2 gg;
    gg.x = (now > ee.x) ? 0.0 : ww.x * 0.5 + hh.x + (double)ss.x;
    gg.y = (now > ee.y) ? 0.0 : ww.y * 0.5 + hh.y + (double)ss.y;
    g[i] = gg;
    longlong2 xx;
    xx.x = now + ss.x;
    xx.y = now + ss.y;
    x[i] = xx;
  }
}

template <int NT>
__device__ double block_sum(double v, double* lds) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = lds[0];
  for (int i = 1; i < NT / 64; ++i) r += lds[i];
  __syncthreads();
  return r;
}

// 3. one 256-thread block per segment (S <= 1024), rows in registers, NRED
//    dependent block reductions, then the writes (the shape of block256x4).
template <int R, int NRED, int W16>
__global__ __launch_bounds__(256) void k_seg(const double* __restrict__ w, const double* __restrict__ h,
                                            const long long* __restrict__ s, const long long* __restrict__ e,
                                            double* __restrict__ g, long long* __restrict__ x, int S,
                                            long long now) {
  __shared__ double lds[4];
  const long long lo = (long long)blockIdx.x * S;
  double wv[R], hv[R];
  long long sv[R];
  unsigned live = 0, valid = 0;
  if (W16) {
    // two consecutive rows per lane per load (S even, lo even)
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const int i = (k * 256 + threadIdx.x) * 2;
      if (i < S) {
        const double2 a = *(const double2*)(w + lo + i);
        const double2 b = *(const double2*)(h + lo + i);
        const longlong2 c = *(const longlong2*)(s + lo + i);
        const longlong2 d = *(const longlong2*)(e + lo + i);
        wv[2 * k] = a.x; wv[2 * k + 1] = a.y;
        hv[2 * k] = b.x; hv[2 * k + 1] = b.y;
        sv[2 * k] = c.x; sv[2 * k + 1] = c.y;
        valid |= 3u << (2 * k);
        if (!(now > d.x)) live |= 1u << (2 * k);
        if (!(now > d.y)) live |= 2u << (2 * k);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * 256 + threadIdx.x;
      wv[k] = hv[k] = 0.0;
      sv[k] = 0;
      if (i < S) {
        wv[k] = w[lo + i];
        hv[k] = h[lo + i];
        sv[k] = s[lo + i];
        valid |= 1u << k;
        if (!(now > e[lo + i])) live |= 1u << k;
      }
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < NRED; ++r) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (live >> k & 1) v += wv[k] * (acc + 1.0) - hv[k];
    acc += block_sum<256>(v, lds) * 1e-30;
  }
  if (W16) {
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const int i = (k * 256 + threadIdx.x) * 2;
      if (i < S) {
        double2 a;
        a.x = wv[2 * k] + acc;
        a.y = wv[2 * k + 1] + acc;
        *(double2*)(g + lo + i) = a;
        longlong2 b;
        b.x = now + sv[2 * k];
        b.y = now + sv[2 * k + 1];
        *(longlong2*)(x + lo + i) = b;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (!(valid >> k & 1)) continue;
      const int i = k * 256 + threadIdx.x;
      g[lo + i] = (live >> k & 1) ? wv[k] + acc : 0.0;
      x[lo + i] = now + sv[k];
    }
  }
}


template <typename T>
__device__ __forceinline__ void st(T* p, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p); else *p = v;
}

// 4. persistent workgroups, software-pipelined over segments: the next
//    segment's rows are loaded into a second register set while the current
//    one is reduced and written.
template <int R, int NRED, bool NT>
__global__ __launch_bounds__(256) void k_pipe(const double* __restrict__ w, const double* __restrict__ h,
                                             const long long* __restrict__ s, const long long* __restrict__ e,
                                             double* __restrict__ g, long long* __restrict__ x, int S, int nseg,
                                             long long now) {
  __shared__ double lds[4];
  double wv[2][R], hv[2][R];
  long long sv[2][R];
  unsigned live[2] = {0, 0};
  auto load = [&](int b, int seg) {
    const long long lo = (long long)seg * S;
    live[b] = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * 256 + threadIdx.x;
      wv[b][k] = hv[b][k] = 0.0;
      sv[b][k] = 0;
      if (seg < nseg && i < S) {
        wv[b][k] = w[lo + i];
        hv[b][k] = h[lo + i];
        sv[b][k] = s[lo + i];
        if (!(now > e[lo + i])) live[b] |= 1u << k;
      }
    }
  };
  auto work = [&](int b, int seg) {
    const long long lo = (long long)seg * S;
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < NRED; ++r) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k)
        if (live[b] >> k & 1) v += wv[b][k] * (acc + 1.0) - hv[b][k];
      acc += block_sum<256>(v, lds) * 1e-30;
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * 256 + threadIdx.x;
      if (i < S) {
        st(g + lo + i, (live[b] >> k & 1) ? wv[b][k] + acc : 0.0, NT);
        st(x + lo + i, now + sv[b][k], NT);
      }
    }
  };
  int seg = blockIdx.x;
  load(0, seg);
  for (; seg < nseg; seg += 2 * gridDim.x) {
    load(1, seg + gridDim.x);
    work(0, seg);
    if (seg + gridDim.x >= nseg) break;
    load(0, seg + 2 * gridDim.x);
    work(1, seg + gridDim.x);
  }
}

// 5. flat stream with non-temporal stores
__global__ __launch_bounds__(256) void k_flat8nt(const double* __restrict__ w, const double* __restrict__ h,
                                                const long long* __restrict__ s, const long long* __restrict__ e,
                                                double* __restrict__ g, long long* __restrict__ x, long long n,
                                                long long now) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double ww = w[i], hh = h[i];
    const long long ss = s[i], ee = e[i];
    __builtin_nontemporal_store((now > ee) ? 0.0 : ww * 0.5 + hh + (double)ss, g + i);
    __builtin_nontemporal_store(now + ss, x + i);
  }
}

// 6. segment kernel with non-temporal stores (k_seg R4 NRED, 8-byte)
template <int R, int NRED>
__global__ __launch_bounds__(256) void k_segnt(const double* __restrict__ w, const double* __restrict__ h,
                                              const long long* __restrict__ s, const long long* __restrict__ e,
                                              double* __restrict__ g, long long* __restrict__ x, int S,
                                              long long now) {
  __shared__ double lds[4];
  const long long lo = (long long)blockIdx.x * S;
  double wv[R], hv[R];
  long long sv[R];
  unsigned live = 0, valid = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = k * 256 + threadIdx.x;
    wv[k] = hv[k] = 0.0;
    sv[k] = 0;
    if (i < S) {
      wv[k] = w[lo + i];
      hv[k] = h[lo + i];
      sv[k] = s[lo + i];
      valid |= 1u << k;
      if (!(now > e[lo + i])) live |= 1u << k;
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < NRED; ++r) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (live >> k & 1) v += wv[k] * (acc + 1.0) - hv[k];
    acc += block_sum<256>(v, lds) * 1e-30;
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (!(valid >> k & 1)) continue;
    const int i = k * 256 + threadIdx.x;
    __builtin_nontemporal_store((live >> k & 1) ? wv[k] + acc : 0.0, g + lo + i);
    __builtin_nontemporal_store(now + sv[k], x + lo + i);
  }
}

template <typename F>
static float time_it(F&& launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const long long N = argc > 1 ? atoll(argv[1]) : 10000000LL;
  const int S = argc > 2 ? atoi(argv[2]) : 1000;
  const int reps = 50;
  double *w, *h, *g;
  long long *s, *e, *x;
  CK(hipMalloc((void**)&w, N * 8));
  CK(hipMalloc((void**)&h, N * 8));
  CK(hipMalloc((void**)&g, N * 8));
  CK(hipMalloc((void**)&s, N * 8));
  CK(hipMalloc((void**)&e, N * 8));
  CK(hipMalloc((void**)&x, N * 8));
  std::vector<double> hw(N);
  for (long long i = 0; i < N; ++i) hw[i] = (double)(i % 997) * 0.001;
  CK(hipMemcpy(w, hw.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(h, hw.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset((void*)s, 0, N * 8));
  CK(hipMemset((void*)e, 0x7f, N * 8));
  const double bytes = 48.0 * N;
  const long long now = 1;
  auto report = [&](const char* name, float ms) {
    printf("%-28s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  for (int grid : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "flat8 grid=%d", grid);
    report(nm, time_it([&] { k_flat8<<<grid, 256>>>(w, h, s, e, g, x, N, now); }, reps));
    snprintf(nm, sizeof nm, "flat16 grid=%d", grid);
    report(nm, time_it([&] {
             k_flat16<<<grid, 256>>>((const double2*)w, (const double2*)h, (const longlong2*)s, (const longlong2*)e,
                                     (double2*)g, (longlong2*)x, N / 2, now);
           }, reps));
  }
  const int nseg = (int)(N / S);
  report("seg R4 red0 w8", time_it([&] { k_seg<4, 0, 0><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  report("seg R4 red1 w8", time_it([&] { k_seg<4, 1, 0><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  report("seg R4 red4 w8", time_it([&] { k_seg<4, 4, 0><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  report("seg R4 red8 w8", time_it([&] { k_seg<4, 8, 0><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  report("segNT R4 red4", time_it([&] { k_segnt<4, 4><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  for (int grid : {512, 768, 1024, 1280}) {
    char nm[64];
    snprintf(nm, sizeof nm, "pipe R4 red4 grid=%d", grid);
    report(nm, time_it([&] { k_pipe<4, 4, false><<<grid, 256>>>(w, h, s, e, g, x, S, nseg, now); }, reps));
    snprintf(nm, sizeof nm, "pipeNT R4 red4 grid=%d", grid);
    report(nm, time_it([&] { k_pipe<4, 4, true><<<grid, 256>>>(w, h, s, e, g, x, S, nseg, now); }, reps));
  }
  report("flat8NT grid=1024", time_it([&] { k_flat8nt<<<1024, 256>>>(w, h, s, e, g, x, N, now); }, reps));
  report("flat8NT grid=2048", time_it([&] { k_flat8nt<<<2048, 256>>>(w, h, s, e, g, x, N, now); }, reps));
  report("seg R4 red0 w16", time_it([&] { k_seg<4, 0, 1><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  report("seg R4 red4 w16", time_it([&] { k_seg<4, 4, 1><<<nseg, 256>>>(w, h, s, e, g, x, S, now); }, reps));
  return 0;
}
