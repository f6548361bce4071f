// dm_records.h — per-chunk / per-resource hand-off records of the in-launch large
// paths (dm_large.hip: one launch with rows resident; dm_flow.hip: one persistent
// launch with a task queue).  A record is kFusedWords u64 words (dm_device.h):
//   0 cnt  1 has  2 wants  3 all.cnt  4 all.has  5 all.wants  6 smin|smax<<32  7 nan
//   8 b.x  9 b.y  10 b.i   11 c.ee  12 c.sgt  13 delta
// stored write-through (st_wt) and loaded with agent-scope loads (ld_wt), the
// MI355X_MICROARCH.md "Valid forms" first-row hand-off (dm_kernel_util.h).
#pragma once
#include "dm_kernel_util.h"

namespace dm {

__device__ __forceinline__ uint64_t bits(double d) { return __builtin_bit_cast(uint64_t, d); }
__device__ __forceinline__ uint64_t bits(long long i) { return (uint64_t)i; }
__device__ __forceinline__ double dbl(uint64_t u) { return __builtin_bit_cast(double, u); }

__device__ __forceinline__ void store_a(uint64_t* r, const AggA& a) {
  st_wt(r + 0, bits(a.cnt));
  st_wt(r + 1, bits(a.h));
  st_wt(r + 2, bits(a.w));
  st_wt(r + 3, bits(a.all.cnt));
  st_wt(r + 4, bits(a.all.h));
  st_wt(r + 5, bits(a.all.w));
  st_wt(r + 6, (uint64_t)(uint32_t)a.smin | ((uint64_t)(uint32_t)a.smax << 32));
  st_wt(r + 7, (uint64_t)(uint32_t)a.nan);
}
__device__ __forceinline__ AggA load_a(const uint64_t* r) {
  AggA a;
  a.cnt = (long long)ld_wt(r + 0);
  a.h = dbl(ld_wt(r + 1));
  a.w = dbl(ld_wt(r + 2));
  a.all.cnt = (long long)ld_wt(r + 3);
  a.all.h = dbl(ld_wt(r + 4));
  a.all.w = dbl(ld_wt(r + 5));
  const uint64_t mm = ld_wt(r + 6);
  a.smin = (int)(uint32_t)mm;
  a.smax = (int)(uint32_t)(mm >> 32);
  a.nan = (int)(uint32_t)ld_wt(r + 7);
  a.nlive = 0;
  return a;
}
__device__ __forceinline__ void store_b(uint64_t* r, const AggB& b) {
  st_wt(r + 8, bits(b.x));
  st_wt(r + 9, bits(b.y));
  st_wt(r + 10, bits(b.i));
}
__device__ __forceinline__ AggB load_b(const uint64_t* r) {
  return AggB{dbl(ld_wt(r + 8)), dbl(ld_wt(r + 9)), (long long)ld_wt(r + 10)};
}
__device__ __forceinline__ void store_c(uint64_t* r, const AggC& c) {
  st_wt(r + 11, bits(c.ee));
  st_wt(r + 12, bits(c.sgt));
}
__device__ __forceinline__ AggC load_c(const uint64_t* r) { return AggC{dbl(ld_wt(r + 11)), (long long)ld_wt(r + 12)}; }

// the totals record's words as broadcast through LDS
__device__ __forceinline__ AggA xt_a(const uint64_t* xt) {
  AggA a;
  a.cnt = (long long)xt[0];
  a.h = dbl(xt[1]);
  a.w = dbl(xt[2]);
  a.all = AggR{(long long)xt[3], dbl(xt[4]), dbl(xt[5])};
  a.smin = (int)(uint32_t)xt[6];
  a.smax = (int)(uint32_t)(xt[6] >> 32);
  a.nan = (int)(uint32_t)xt[7];
  a.nlive = 0;
  return a;
}
__device__ __forceinline__ AggB xt_b(const uint64_t* xt) { return AggB{dbl(xt[8]), dbl(xt[9]), (long long)xt[10]}; }
__device__ __forceinline__ AggC xt_c(const uint64_t* xt) { return AggC{dbl(xt[11]), (long long)xt[12]}; }

// per large resource sync words (kFusedSync): arrive counters 0..3 on one line, then
// the flag of phase k replicated kFusedFlagCopies times, each replica on its own line
__device__ __forceinline__ int flag_at(int phase) { return 32 + phase * kFusedFlagCopies * 32; }

// Bounded poll of one flag word by one lane; false when it gave up.
__device__ __forceinline__ bool wait_flag(uint32_t* flag, uint32_t epoch, uint32_t limit, uint32_t* err) {
  for (uint32_t spins = 0; __hip_atomic_load((gu32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch;
       ++spins) {
    if (spins >= limit) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  return true;
}

// Last arriver, wave 0: publish the totals record (lane 0 stored it), then every
// replica of the phase's flag (lanes 0..kFusedFlagCopies-1, one store instruction).
__device__ __forceinline__ void publish_flag(uint32_t* flags, uint32_t epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // totals landed before the flag
  if (threadIdx.x < kFusedFlagCopies)
    __hip_atomic_store((gu32*)(flags + threadIdx.x * 32), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dm
