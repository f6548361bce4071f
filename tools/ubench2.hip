// ubench2.hip — what the segmented tick's reductions cost, and what hides them.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench2 tools/ubench2.hip
// Same traffic as the tick (read wants/has/sub/expiry, write gets/expiry = 48 B
// per row), one workgroup (or one wave, G = 64) per segment of S rows, NRED
// dependent group reductions between the loads and the gets stores, then one
// trailing reduction (the tick's sum of gets - has).  Knobs:
//   G, R     threads per segment and rows per thread (G*R >= S)
//   W16      two adjacent rows per lane per load/store (dwordx4)
//   EARLY    expiry output stored right after the loads (it needs no reduction)
//   OCC      amdgpu_waves_per_eu lower bound (0 = compiler's choice)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef long long lv2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t err_ = (x);                                                            \
    if (err_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_));    \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)


template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, true);
  hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rl(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return (rl(v, 0) + rl(v, 16)) + (rl(v, 32) + rl(v, 48));
}
template <int G>
__device__ __forceinline__ double group_sum(double v, double* lds) {
  v = wave_sum(v);
  if constexpr (G == 64) {
    return v;
  } else {
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = lds[0];
    for (int i = 1; i < G / 64; ++i) r += lds[i];
    __syncthreads();
    return r;
  }
}

template <int G, int R, int NRED, int W16, int EARLY>
__device__ __forceinline__ void seg_body(const double* __restrict__ w, const double* __restrict__ h,
                                         const long long* __restrict__ s, const long long* __restrict__ e,
                                         double* __restrict__ g, long long* __restrict__ x, double* __restrict__ out,
                                         int seg, int S, int t, double* lds, long long now) {
  const long long lo = (long long)seg * S;
  const double* wb = w + lo;
  const double* hb = h + lo;
  const long long* sb = s + lo;
  const long long* eb = e + lo;
  double* gb = g + lo;
  long long* xb = x + lo;
  double wv[R], hv[R];
  int sv[R];
  unsigned live = 0, valid = 0;
  const long long xo = now + 300000000000LL;
  if (W16) {
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const unsigned i = (unsigned)(k * G + t) * 2;
      wv[2 * k] = wv[2 * k + 1] = hv[2 * k] = hv[2 * k + 1] = 0.0;
      sv[2 * k] = sv[2 * k + 1] = 0;
      if ((int)i < S) {
        const double2 a = *(const double2*)(wb + i);
        const double2 b = *(const double2*)(hb + i);
        const longlong2 c = *(const longlong2*)(sb + i);
        const longlong2 d = *(const longlong2*)(eb + i);
        wv[2 * k] = a.x; wv[2 * k + 1] = a.y;
        hv[2 * k] = b.x; hv[2 * k + 1] = b.y;
        sv[2 * k] = (int)c.x; sv[2 * k + 1] = (int)c.y;
        valid |= 3u << (2 * k);
        const bool l0 = !(now > d.x), l1 = !(now > d.y);
        live |= (l0 ? 1u : 0u) << (2 * k);
        live |= (l1 ? 2u : 0u) << (2 * k);
        if (EARLY) {
          lv2 o;
          o.x = l0 ? xo : INT64_MIN;
          o.y = l1 ? xo : INT64_MIN;
          __builtin_nontemporal_store(o, (lv2*)(xb + i));
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const unsigned i = (unsigned)(k * G + t);
      wv[k] = hv[k] = 0.0;
      sv[k] = 0;
      if ((int)i < S) {
        wv[k] = wb[i];
        hv[k] = hb[i];
        sv[k] = (int)sb[i];
        const bool l = !(now > eb[i]);
        valid |= 1u << k;
        live |= (l ? 1u : 0u) << k;
        if (EARLY) __builtin_nontemporal_store(l ? xo : (long long)INT64_MIN, xb + i);
      }
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < NRED; ++r) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (live >> k & 1) v += (wv[k] < acc + 1.0 ? wv[k] : hv[k]) * (double)sv[k];
    acc += group_sum<G>(v, lds) * 1e-30;
  }
  double d = 0.0;
  if (W16) {
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const unsigned i = (unsigned)(k * G + t) * 2;
      if ((int)i < S) {
        dv2 a;
        a.x = (live >> (2 * k) & 1) ? wv[2 * k] + acc : 0.0;
        a.y = (live >> (2 * k + 1) & 1) ? wv[2 * k + 1] + acc : 0.0;
        d += a.x - hv[2 * k] + a.y - hv[2 * k + 1];
        __builtin_nontemporal_store(a, (dv2*)(gb + i));
        if (!EARLY) {
          lv2 o;
          o.x = (live >> (2 * k) & 1) ? xo : INT64_MIN;
          o.y = (live >> (2 * k + 1) & 1) ? xo : INT64_MIN;
          __builtin_nontemporal_store(o, (lv2*)(xb + i));
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (!(valid >> k & 1)) continue;
      const unsigned i = (unsigned)(k * G + t);
      const bool l = live >> k & 1;
      const double gg = l ? wv[k] + acc : 0.0;
      d += gg - hv[k];
      __builtin_nontemporal_store(gg, gb + i);
      if (!EARLY) __builtin_nontemporal_store(l ? xo : (long long)INT64_MIN, xb + i);
    }
  }
  d = group_sum<G>(d, lds);
  if (t == 0) out[seg] = d;
}

#define DEF_SEG(NAME, G, OCC)                                                                              \
  template <int R, int NRED, int W16, int EARLY>                                                          \
  __global__ __launch_bounds__(G == 64 ? 256 : G) __attribute__((amdgpu_waves_per_eu(OCC)))             \
  void NAME(const double* __restrict__ w, const double* __restrict__ h, const long long* __restrict__ s,   \
            const long long* __restrict__ e, double* __restrict__ g, long long* __restrict__ x,            \
            double* __restrict__ out, int S, int nseg, long long now) {                                   \
    __shared__ double lds[G / 64 + 1];                                                                    \
    if (G == 64) {                                                                                        \
      const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);                                                \
      if (seg >= nseg) return;                                                                            \
      seg_body<64, R, NRED, W16, EARLY>(w, h, s, e, g, x, out, seg, S, threadIdx.x & 63, lds, now);       \
    } else {                                                                                              \
      seg_body<G, R, NRED, W16, EARLY>(w, h, s, e, g, x, out, blockIdx.x, S, threadIdx.x, lds, now);      \
    }                                                                                                     \
  }

DEF_SEG(k256, 256, 1)
DEF_SEG(k256o6, 256, 6)
DEF_SEG(k256o8, 256, 8)
DEF_SEG(k512, 512, 1)
DEF_SEG(k1024, 1024, 1)
DEF_SEG(k64, 64, 1)

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
  const int reps = 30;
  const int nseg = (int)(N / S);
  double *w, *h, *g, *out;
  long long *s, *e, *x;
  CK(hipMalloc((void**)&w, N * 8));
  CK(hipMalloc((void**)&h, N * 8));
  CK(hipMalloc((void**)&g, N * 8));
  CK(hipMalloc((void**)&s, N * 8));
  CK(hipMalloc((void**)&e, N * 8));
  CK(hipMalloc((void**)&x, N * 8));
  CK(hipMalloc((void**)&out, (size_t)nseg * 8));
  std::vector<double> hw(N);
  for (long long i = 0; i < N; ++i) hw[i] = (double)(i % 997) * 0.001;
  CK(hipMemcpy(w, hw.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(h, hw.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset((void*)s, 0, N * 8));
  CK(hipMemset((void*)e, 0x7f, N * 8));
  const double bytes = 48.0 * N;
  const long long now = 1;
  auto report = [&](const char* name, float ms) {
    printf("%-34s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
#define RUN(K, G, R, NRED, W16, EARLY)                                                                    \
  do {                                                                                                    \
    const int grid = (G == 64) ? (nseg + 3) / 4 : nseg;                                                   \
    report(#K " R" #R " red" #NRED " w16=" #W16 " early=" #EARLY, time_it([&] {                         \
             K<R, NRED, W16, EARLY><<<grid, (G == 64 ? 256 : G)>>>(w, h, s, e, g, x, out, S, nseg, now);  \
           }, reps));                                                                                     \
  } while (0)
  RUN(k256, 256, 4, 0, 0, 0);
  RUN(k256, 256, 4, 3, 0, 0);
  RUN(k256, 256, 4, 3, 0, 1);
  RUN(k256, 256, 4, 3, 1, 0);
  RUN(k256, 256, 4, 3, 1, 1);
  RUN(k256o6, 256, 4, 3, 0, 0);
  RUN(k256o8, 256, 4, 3, 0, 0);
  RUN(k256o8, 256, 4, 3, 0, 1);
  RUN(k256o8, 256, 4, 3, 1, 1);
  RUN(k512, 512, 2, 3, 0, 0);
  RUN(k512, 512, 2, 3, 0, 1);
  RUN(k512, 512, 2, 3, 1, 1);
  RUN(k1024, 1024, 1, 3, 0, 0);
  RUN(k1024, 1024, 1, 3, 0, 1);
  RUN(k1024, 1024, 2, 3, 1, 1);
  RUN(k64, 64, 16, 3, 0, 0);
  RUN(k64, 64, 16, 3, 0, 1);
  RUN(k64, 64, 16, 3, 1, 1);
  RUN(k256, 256, 4, 1, 0, 0);
  RUN(k256, 256, 4, 1, 0, 1);
  // occupancy emulated with unused dynamic LDS: WG per CU = 160 KiB / shmem
  for (int wgs : {3, 4, 5, 6, 8}) {
    const size_t sh = 163840 / wgs - 256;
    char nm[64];
    snprintf(nm, sizeof nm, "k256 R4 red3 wg/cu=%d", wgs);
    report(nm, time_it([&] { k256<4, 3, 0, 0><<<nseg, 256, sh>>>(w, h, s, e, g, x, out, S, nseg, now); }, reps));
    snprintf(nm, sizeof nm, "k256 R4 red3 early wg/cu=%d", wgs);
    report(nm, time_it([&] { k256<4, 3, 0, 1><<<nseg, 256, sh>>>(w, h, s, e, g, x, out, S, nseg, now); }, reps));
  }
  return 0;
}
