// ubench3.hip — pure-HBM behaviour of the group kernel's load shape (C3 size):
// serial (one row-block of 4 columns per memory round trip) vs all loads in
// flight at once, against the placement of the 6 column arrays (stagger).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench3 tools/ubench3.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t err_ = (x);                                                         \
    if (err_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      exit(1);                                                                     \
    }                                                                              \
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
__device__ __forceinline__ double block_sum(double v, double* lds) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  v = (rl(v, 0) + rl(v, 16)) + (rl(v, 32) + rl(v, 48));
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = lds[0] + lds[1] + lds[2] + lds[3];
  __syncthreads();
  return r;
}

struct Cols {
  const double* w;
  const double* h;
  const long long* s;
  const long long* e;
  double* g;
  long long* x;
};

template <int R, int MODE>  // MODE 0: serial row-blocks, 1: all loads at once, 2: pairs of row-blocks
__global__ __launch_bounds__(256) void k_seg(Cols c, double* out, int S, long long now) {
  __shared__ double lds[4];
  const long long lo = (long long)blockIdx.x * S;
  const int t = threadIdx.x;
  double wv[R], hv[R];
  int sv[R];
  long long ev[R];
  unsigned live = 0, valid = 0;
  if (MODE == 0) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * 256 + t;
      wv[k] = hv[k] = 0.0;
      sv[k] = 0;
      if (i < S) {
        wv[k] = c.w[lo + i];
        hv[k] = c.h[lo + i];
        sv[k] = (int)c.s[lo + i];
        valid |= 1u << k;
        if (!(now > c.e[lo + i])) live |= 1u << k;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * 256 + t;
      const unsigned u = (unsigned)(i < S ? i : S - 1);
      wv[k] = c.w[lo + u];
      hv[k] = c.h[lo + u];
      sv[k] = (int)c.s[lo + u];
      ev[k] = c.e[lo + u];
      if (MODE == 2 && (k & 1)) __builtin_amdgcn_s_waitcnt(0x0f70 & ~0xf);  // vmcnt(0) after each pair
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const unsigned vk = (k * 256 + t < S) ? 1u : 0u;
      valid |= vk << k;
      live |= (vk & (now > ev[k] ? 0u : 1u)) << k;
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (live >> k & 1) v += (wv[k] < acc + 1.0 ? wv[k] : hv[k]) * (double)sv[k];
    acc += block_sum(v, lds) * 1e-30;
  }
  double d = 0.0;
  const long long xo = now + 300000000000LL;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (!(valid >> k & 1)) continue;
    const int i = k * 256 + t;
    const bool l = live >> k & 1;
    const double gg = l ? wv[k] + acc : 0.0;
    d += gg - hv[k];
    __builtin_nontemporal_store(gg, c.g + lo + i);
    __builtin_nontemporal_store(l ? xo : (long long)INT64_MIN, c.x + lo + i);
  }
  d = block_sum(d, lds);
  if (t == 0) out[blockIdx.x] = d;
}

int main(int argc, char** argv) {
  const long long N = argc > 1 ? atoll(argv[1]) : 100000000LL;
  const int S = 1000;
  const int nseg = (int)(N / S);
  const long long col = N * 8;
  const long long maxstag = 1 << 24;
  char* pool;
  CK(hipMalloc((void**)&pool, 6 * (col + maxstag) + 4096));
  CK(hipMemset(pool, 0, 6 * (col + maxstag)));
  double* out;
  CK(hipMalloc((void**)&out, (size_t)nseg * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const long long now = 1;
  const long long stags[] = {0, 256, 4096, 4096 + 256, 65536 + 4096 + 256, 1 << 20, (1 << 20) + 12544};
  for (long long st : stags) {
    Cols c;
    char* p = pool;
    auto take = [&](int k) {
      char* q = p + k * (col + st);
      return q;
    };
    c.w = (const double*)take(0);
    c.h = (const double*)take(1);
    c.s = (const long long*)take(2);
    c.e = (const long long*)take(3);
    c.g = (double*)take(4);
    c.x = (long long*)take(5);
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&] {
        if (mode == 0) k_seg<4, 0><<<nseg, 256>>>(c, out, S, now);
        if (mode == 1) k_seg<4, 1><<<nseg, 256>>>(c, out, S, now);
        if (mode == 2) k_seg<4, 2><<<nseg, 256>>>(c, out, S, now);
      };
      for (int i = 0; i < 3; ++i) launch();
      const int reps = 10;
      CK(hipEventRecord(a));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= reps;
      printf("stagger %8lld mode %d  %8.1f us  %7.1f GB/s\n", st, mode, ms * 1e3, 48.0 * N / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
