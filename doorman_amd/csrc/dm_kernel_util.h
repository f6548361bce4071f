// dm_kernel_util.h — device helpers shared by the gfx950 kernels (dm_kernels.hip,
// dm_round.hip): Go float semantics, DPP/readlane wave reductions, the
// per-resource aggregates and the FairShare per-row stages.
#pragma once
#include <hip/hip_runtime.h>

#include "dm_device.h"

namespace dm {

// --------------------------------------------------------------------------
// helpers
// --------------------------------------------------------------------------
__device__ __forceinline__ double minF(double l, double r) { return l > r ? r : l; }  // algorithm.go:50-55

struct Res {
  int32_t kind;
  int32_t learning;
  double C;           // Resource.capacity() (resource.go:62-70)
  int64_t exp_out;    // now + lease_length (store.go:161)
  int64_t follow_exp; // the expiry of the resource's follower rows (dm_device.h)
  int32_t xstate;     // DevParams::expl (dm_device.h): 1 = rows may carry explicit expiries (wave-uniform,
                      // so no row's expiry load waits on its subclients word); s0 + 1 >= 2 = dense
  // the store's running sums, loaded with the config so that no global load
  // waits behind the first reduction's barrier
  long long agg_count;
  double agg_has;
  double agg_wants;
};

__device__ __forceinline__ bool any_explicit(const Res& r) { return r.xstate == 1; }
__device__ __forceinline__ int dense_subclients(const Res& r) { return r.xstate >= 2 ? r.xstate - 1 : 0; }

__device__ __forceinline__ Res load_res(const DevParams& p, int seg) {
  Res r;
  const ResCfg c = p.cfg[seg];
  r.kind = c.kind;
  r.learning = c.learning_end_ns > p.now;  // resource.go:108 learningModeEndTime.After(now)
  r.C = (c.parent_expiry_ns < p.now) ? 0.0 : c.capacity;  // expiryTime.Before(now)
  r.exp_out = p.now + (int64_t)c.lease_len_s * kNs;
  const ResAgg g = p.agg[seg];
  r.follow_exp = g.follow_exp;
  r.xstate = p.expl[seg];
  if (!p.recompute) {
    r.agg_count = g.count;
    r.agg_has = g.sum_has;
    r.agg_wants = g.sum_wants;
  } else {
    r.agg_count = 0;
    r.agg_has = 0.0;
    r.agg_wants = 0.0;
  }
  return r;
}

template <typename T>
__device__ __forceinline__ T shfl_any(const T& v, int lane) {
  int src[sizeof(T) / 4], dst[sizeof(T) / 4];
  __builtin_memcpy(src, &v, sizeof(T));
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = __shfl(src[i], lane, 64);
  T r;
  __builtin_memcpy(&r, dst, sizeof(T));
  return r;
}

// A value every lane holds identically (an LDS broadcast, a combine of readlanes),
// moved to SGPRs: uniform values that stay in VGPRs through a kernel's later
// passes cost a register per dword per lane and with it occupancy.
template <typename T>
__device__ __forceinline__ T uniform(const T& v) {
  static_assert(sizeof(T) % 4 == 0, "4-byte granular");
  int src[sizeof(T) / 4], dst[sizeof(T) / 4];
  __builtin_memcpy(src, &v, sizeof(T));
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = __builtin_amdgcn_readfirstlane(src[i]);
  T r;
  __builtin_memcpy(&r, dst, sizeof(T));
  return r;
}

// DPP lane permute of every dword of v (a VALU operand modifier: no LDS trip).
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_any(const T& v) {
  static_assert(sizeof(T) % 4 == 0, "4-byte granular");
  int src[sizeof(T) / 4], dst[sizeof(T) / 4];
  __builtin_memcpy(src, &v, sizeof(T));
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i)
    dst[i] = __builtin_amdgcn_update_dpp(0, src[i], CTRL, 0xF, 0xF, true);
  T r;
  __builtin_memcpy(&r, dst, sizeof(T));
  return r;
}

template <typename T>
__device__ __forceinline__ T readlane_any(const T& v, int lane) {
  int src[sizeof(T) / 4], dst[sizeof(T) / 4];
  __builtin_memcpy(src, &v, sizeof(T));
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = __builtin_amdgcn_readlane(src[i], lane);
  T r;
  __builtin_memcpy(&r, dst, sizeof(T));
  return r;
}

// Wave reduction: a DPP butterfly inside each 16-lane row (xor 1, xor 2, half
// mirror, mirror: partner lanes compute a+b and b+a, so every lane of a row holds
// the same row total), then the four row totals combined in a fixed order from
// scalar readlanes.  Requires all 64 lanes active.
// Sub-wave groups (G = 8: half a DPP row, G = 16: one DPP row, G = 32: half a
// wave) reduce within themselves: every lane of the group gets its group's total.
template <int G, typename T, typename Op>
__device__ __forceinline__ T wave_reduce_g(T v, Op op) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "sub-wave group");
  v = op(v, dpp_any<0xB1>(v));   // quad_perm [1,0,3,2]: 2-lane totals
  if constexpr (G == 2) return v;
  v = op(v, dpp_any<0x4E>(v));   // quad_perm [2,3,0,1]: 4-lane totals
  if constexpr (G == 4) return v;
  v = op(v, dpp_any<0x141>(v));  // row_half_mirror: 8-lane totals
  if constexpr (G == 8) return v;
  v = op(v, dpp_any<0x140>(v));  // row_mirror
  if constexpr (G == 16) {
    return v;
  } else {
    const T r0 = readlane_any(v, 0), r1 = readlane_any(v, 16), r2 = readlane_any(v, 32), r3 = readlane_any(v, 48);
    if constexpr (G == 32) {
      const T lo = op(r0, r1), hi = op(r2, r3);
      return (threadIdx.x & 32) ? hi : lo;
    } else {
      return op(op(r0, r1), op(r2, r3));
    }
  }
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
  return wave_reduce_g<64>(v, op);
}

// Group reduction (G = 64: one wave; G >= 256: the waves' totals through LDS).
// Every thread combines the wave totals in the same fixed order, so all threads
// (and all workgroups reducing the same inputs) agree bit for bit.
// REUSE = false: the LDS slots are written once per workgroup (group_segment
// gives every reduction its own slots), so the barrier that protects them from
// the next reduction's writes is dropped.
template <int G, typename T, typename Op, bool REUSE = true>
__device__ __forceinline__ T group_reduce(T v, Op op, T* lds) {
  v = wave_reduce_g<(G < 64 ? G : 64)>(v, op);
  if constexpr (G <= 64) {
    (void)lds;
    return v;
  } else {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds[w] = v;
    __syncthreads();
    T r = lds[0];
#pragma unroll 3
    for (int i = 1; i < G / 64; ++i) {
      const T x = lds[i];
      r = op(r, x);
    }
    if constexpr (REUSE) __syncthreads();
    return uniform(r);
  }
}

// As group_reduce, but only thread 0 combines the waves' totals: the result is
// defined in thread 0 only (partials that one thread stores).  The other threads skip
// the LDS reads and the combine; the slots are written once (no trailing barrier).
template <int G, typename T, typename Op>
__device__ __forceinline__ T group_reduce_t0(T v, Op op, T* lds) {
  static_assert(G >= 128, "workgroups of two or more waves");
  v = wave_reduce_g<64>(v, op);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    T r = lds[0];
#pragma unroll
    for (int i = 1; i < G / 64; ++i) r = op(r, lds[i]);
    v = r;
  }
  return v;
}

struct AggR {  // every row: the store's sums rebuilt by Assign (recompute mode)
  long long cnt;
  double h;
  double w;
};
struct OpR {
  __device__ AggR operator()(AggR a, AggR b) const {
    AggR r;
    r.cnt = a.cnt + b.cnt;
    r.h = a.h + b.h;
    r.w = a.w + b.w;
    return r;
  }
};

struct AggA {
  long long cnt;  // leases Clean releases (expired rows)
  double h;
  double w;
  AggR all;       // filled in recompute mode only
  int smin;       // live rows' subclients range and any NaN wants
  int smax;
  int nan;
  int nlive;      // live rows (group kernels: the dense state needs all of them)
};
struct OpA {
  __device__ AggA operator()(AggA a, AggA b) const {
    AggA r;
    r.cnt = a.cnt + b.cnt;
    r.h = a.h + b.h;
    r.w = a.w + b.w;
    r.all = a.all;
    r.smin = a.smin < b.smin ? a.smin : b.smin;
    r.smax = a.smax > b.smax ? a.smax : b.smax;
    r.nan = a.nan | b.nan;
    r.nlive = a.nlive + b.nlive;
    return r;
  }
};
__device__ __forceinline__ AggA zeroA() {
  AggA a;
  a.cnt = 0;
  a.h = 0.0;
  a.w = 0.0;
  a.all = AggR{0, 0.0, 0.0};
  a.smin = INT32_MAX;
  a.smax = INT32_MIN;
  a.nan = 0;
  a.nlive = 0;
  return a;
}

struct AggB {
  double x;    // FS: extra (E)          PS: extraCapacity
  double y;    //                        PS: extraNeed
  long long i; // FS: wantExtra (W)
};
struct OpB {
  __device__ AggB operator()(AggB a, AggB b) const {
    AggB r;
    r.x = a.x + b.x;
    r.y = a.y + b.y;
    r.i = a.i + b.i;
    return r;
  }
};

struct AggC {
  double ee;      // extraExtra
  long long sgt;  // sum of subclients of wantExtraClients above T
};
struct OpC {
  __device__ AggC operator()(AggC a, AggC b) const {
    AggC r;
    r.ee = a.ee + b.ee;
    r.sgt = a.sgt + b.sgt;
    return r;
  }
};

struct TMin {
  double t;
  int found;
  int pad;
};
struct OpTMin {
  __device__ TMin operator()(TMin a, TMin b) const {
    const bool take_b = b.found && (!a.found || b.t < a.t);
    TMin r;
    r.t = take_b ? b.t : a.t;
    r.found = a.found | b.found;
    r.pad = 0;
    return r;
  }
};
__device__ __forceinline__ void tmin_add(TMin& m, double T) {
  const bool take = !m.found || T < m.t;
  m.t = take ? T : m.t;
  m.found = 1;
}

struct SumD {
  double v;
};
struct OpSumD {
  __device__ SumD operator()(SumD a, SumD b) const { return SumD{a.v + b.v}; }
};
struct SumDN {  // the Assign delta plus the live rows (group kernels with the dense state)
  double v;
  int n;
  int pad;
};
struct OpSumDN {
  __device__ SumDN operator()(SumDN a, SumDN b) const { return SumDN{a.v + b.v, a.n + b.n, 0}; }
};

template <int G>
struct Lds {  // one slot per wave (unused by groups of one wave or less)
  static constexpr int W = G >= 64 ? G / 64 : 1;
  AggA a[W];
  AggR r[W];
  AggB b[W];
  AggC c[W];
  TMin t[W];
  SumD d[W];
  SumDN dn[W];
};

// Cleaned store sums from pass A (store.go:169-181 applied to the snapshot).
struct Clean {
  long long count;
  double sum_has;
  double sum_wants;
};
__device__ __forceinline__ Clean clean_from(const DevParams& p, const Res& rs, const AggA& a) {
  // store sums (running, or rebuilt from every row) minus the leases Clean releases
  Clean c;
  if (p.recompute) {
    c.count = a.all.cnt - a.cnt;
    c.sum_has = a.all.h - a.h;
    c.sum_wants = a.all.w - a.w;
  } else {
    c.count = rs.agg_count - a.cnt;
    c.sum_has = rs.agg_has - a.h;
    c.sum_wants = rs.agg_wants - a.w;
  }
  return c;
}

// dense_next (group kernels only): s0 > 0 when after this writeback tick every row of
// the resource is a live follower with subclients s0 (the expl byte becomes s0 + 1).
__device__ __forceinline__ void write_resource(const DevParams& p, int seg, const Res& rs, const Clean& c,
                                               double delta, int dense_next = 0) {
  ResAgg r;
  r.count = c.count;
  r.sum_wants = c.sum_wants;
  r.sum_has = c.sum_has + delta;  // the tick's Assigns: sumHas += gets - has (store.go:156)
  r.follow_exp = p.writeback ? rs.exp_out : rs.follow_exp;  // a writeback tick's leases follow exp_out
  p.res[seg] = r;
  if (p.pub) {  // performRequests' band of the resource (server.go:234-255), as dm_publish_totals
    double2 v;
    v.x = r.sum_wants;
    v.y = __longlong_as_double(r.count);
    p.pub[1 + seg] = v;
    if (r.sum_wants > 0.0 && (r.count < 1 || r.count > kSubMax))  // the root's validation (:863-866)
      atomicOr((unsigned int*)p.pub + (p.pub_word < 0 ? 0 : p.pub_word), r.count < 1 ? kHierInvalid : kHierCountRange);
    if (seg == p.pub_first) {  // the next tick's flags start clear
      if (p.pub_word < 0) p.pub_clear[0] = double2{0.0, 0.0};
      else ((uint32_t*)p.pub_clear)[p.pub_word] = 0u;
    }
  }
  if (p.writeback) {  // ... and none keeps an explicit expiry
    const int had = rs.xstate;
    const int want = dense_next ? dense_next + 1 : 0;
    if (had != want) p.expl[seg] = (uint8_t)want;
  }
}

// ---- the subclients column's expiry encoding (dm_device.h) ----
__device__ __forceinline__ int sub_value(int32_t raw) { return (uint32_t)raw == kSubReleased ? 0 : (raw & 0x7FFFFFFF); }
__device__ __forceinline__ bool sub_released(int32_t raw) { return (uint32_t)raw == kSubReleased; }
__device__ __forceinline__ bool sub_explicit(int32_t raw) { return raw < 0 && (uint32_t)raw != kSubReleased; }
// A row's expiry, for kernels off the tick's hot path (one dependent load at most).
__device__ __forceinline__ int64_t row_expiry(const DevParams& p, int64_t row, int32_t raw, int64_t follow_exp) {
  return sub_released(raw) ? kReleased : (raw < 0 ? p.expiry[row] : follow_exp);
}
// Element i of a column from a wave-uniform base: a 32-bit byte offset, so the
// access can take the scalar-base form (one offset VGPR shared by every column of
// the same width instead of a 64-bit address per column and row).  i * sizeof(T)
// must fit 32 bits (rows within one resource or chunk).
template <typename T>
__device__ __forceinline__ T* col_at(T* base, uint32_t i) {
  return (T*)((char*)base + (uint32_t)(i * (uint32_t)sizeof(T)));
}
template <typename T>
__device__ __forceinline__ const T* col_at(const T* base, uint32_t i) {
  return (const T*)((const char*)base + (uint32_t)(i * (uint32_t)sizeof(T)));
}

// Store a decided live row (row0 + i; row0 wave-uniform where the caller can): its
// gets, and in a writeback tick it becomes a follower (only an explicit row's
// subclients word changes); otherwise its expiry.
template <bool NT = true>
__device__ __forceinline__ void put_live(const DevParams& p, int64_t row0, uint32_t i, double g, const Res& rs,
                                         int32_t raw) {
  if constexpr (NT) __builtin_nontemporal_store(g, col_at(p.out_gets + row0, i));
  else *col_at(p.out_gets + row0, i) = g;
  if (p.writeback) {
    if (raw < 0) *col_at(p.out_sub + row0, i) = raw & 0x7FFFFFFF;
  } else {
    __builtin_nontemporal_store((int64_t)rs.exp_out, col_at(p.out_expiry + row0, i));
  }
}
// Store a row Clean released: no lease; in a writeback tick the row is zeroed and
// marked released (once: an already released row is left alone).
template <bool NT = true>
__device__ __forceinline__ void put_released(const DevParams& p, int64_t row0, uint32_t i, int32_t raw) {
  if constexpr (NT) __builtin_nontemporal_store(0.0, col_at(p.out_gets + row0, i));
  else *col_at(p.out_gets + row0, i) = 0.0;
  if (p.writeback) {
    if (!sub_released(raw)) {
      *col_at(p.out_wants + row0, i) = 0.0;
      *col_at(p.out_sub + row0, i) = (int32_t)kSubReleased;
    }
  } else {
    __builtin_nontemporal_store((int64_t)kReleased, col_at(p.out_expiry + row0, i));
  }
}

// FairShare per-row stage (algorithm.go:115-181).  Returns true when the lease is
// decided here (gets in *g); otherwise fills T = deservedExtra + deservedShare.
__device__ __forceinline__ bool fs_stage01(double w, double h, long long s, double C, double sum_has, double eq,
                                           double E, long long Wc, double* g, double* T) {
  const double ds = eq * (double)s;              // :126 deservedShare
  const double avail = C - sum_has + h;          // :120 available
  if (w <= ds) {                                 // :131
    *g = minF(w, avail);
    return true;
  }
  const long long Wi = Wc + s - (w > ds ? s : 0);  // :148,168 wantExtra (self counted once)
  const double dE = (E / (double)Wi) * (double)s;  // :175 deservedExtra
  if (w < ds + dE) {                               // :179
    *g = minF(w, avail);
    return true;
  }
  *T = dE + ds;
  return false;
}

// Uniform-subclient FairShare: every per-row quantity of algorithm.go:123-204
// that does not depend on the row's own wants/has is a per-resource constant
// (deservedShare, deservedExtra, T, and the two possible deservedExtraExtra).
struct FsU {
  double ds, dE, T, dee_gt, dee_eq;
};
__device__ __forceinline__ FsU make_fsu(double eq, long long s0, double E, long long Wc, AggC c) {
  FsU f;
  f.ds = eq * (double)s0;                      // :126
  f.dE = (E / (double)Wc) * (double)s0;        // :175 (wantExtra == W for every row that gets here)
  f.T = f.dE + f.ds;                           // :197 deservedExtra + deservedShare
  f.dee_gt = (c.ee / (double)(s0 + c.sgt - s0)) * (double)s0;  // :203, row above T (excluded, :193)
  f.dee_eq = (c.ee / (double)(s0 + c.sgt)) * (double)s0;       // :203, row exactly at T
  return f;
}
__device__ __forceinline__ double fs_uniform_row(double w, double h, double C, double sum_has, const FsU& f) {
  const double avail = C - sum_has + h;  // :120
  if (w <= f.ds) return minF(w, avail);  // :131
  if (w < f.ds + f.dE) return minF(w, avail);  // :179
  return minF(f.ds + f.dE + (w > f.T ? f.dee_gt : f.dee_eq), avail);  // :204
}

// FairShare round 2 result for a row given the resource's sums at its T (:189-204).
__device__ __forceinline__ double fs_stage2(double w, double h, long long s, double C, double sum_has, double eq,
                                            double E, long long Wc, double T, const AggC& c) {
  const double ds = eq * (double)s;
  const double avail = C - sum_has + h;
  const long long Wi = Wc + s - (w > ds ? s : 0);
  const double dE = (E / (double)Wi) * (double)s;
  const long long wee = s + c.sgt - ((w > ds && w > T) ? s : 0);  // :189,200 (self excluded, :193)
  const double dEE = (c.ee / (double)wee) * (double)s;             // :203
  return minF(ds + dE + dEE, avail);                               // :204
}

// --------------------------------------------------------------------------
// In-launch hand-off between workgroups (MI355X_MICROARCH.md, "Valid forms",
// first table row): the payload is stored write-through (8- or 4-B agent-scope
// atomic stores, sc1: no release fence, so no L2 write-back of the workgroup's
// other dirty lines), the storing wave drains (s_waitcnt vmcnt(0)) before its
// arrive, and every load of handed-off bytes is an agent-scope atomic load (sc1,
// L1 bypassed) issued after the arrive returned / the flag matched.
// --------------------------------------------------------------------------
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

__device__ __forceinline__ void st_wt(uint64_t* a, uint64_t v) {
  __hip_atomic_store((gu64*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(double* a, double v) { st_wt((uint64_t*)a, __builtin_bit_cast(uint64_t, v)); }
__device__ __forceinline__ void st_wt(int64_t* a, int64_t v) { st_wt((uint64_t*)a, (uint64_t)v); }
__device__ __forceinline__ void st_wt(int32_t* a, int32_t v) {
  __hip_atomic_store((gu32*)a, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_wt(const uint64_t* a) {
  return __hip_atomic_load((gu64*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* a) { return __builtin_bit_cast(double, ld_wt((const uint64_t*)a)); }
__device__ __forceinline__ int64_t ld_wt(const int64_t* a) { return (int64_t)ld_wt((const uint64_t*)a); }
__device__ __forceinline__ int32_t ld_wt(const int32_t* a) {
  return (int32_t)__hip_atomic_load((gu32*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by wave 0 only, after lane 0 stored the workgroup's partial write-through:
// lane 0 drains its stores and arrives at counter `ctr` (one of `nch` arrivals);
// returns, uniformly over the wave, whether this workgroup arrived last.  The last
// arriver resets the counter for the next launch.  The other waves of the
// workgroup need not wait: they may have exited already.
__device__ __forceinline__ bool arrive_last(uint32_t* ctr, int nch) {
  uint32_t last = 0;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial's stores have landed
    const uint32_t old = __hip_atomic_fetch_add((gu32*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (uint32_t)nch - 1 ? 1u : 0u;
    if (last) __hip_atomic_store((gu32*)ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return __builtin_amdgcn_readfirstlane(last) != 0;
}

// A large resource's state once its pass-A totals are known (all chunks agree).
struct SegState {
  AggA a;
  Clean cl;
  Res rs;
  int general;  // FairShare with heterogeneous subclients / NaN wants -> k_general
};

__device__ __forceinline__ SegState seg_state_of(const DevParams& p, int seg, const AggA& a) {
  SegState st;
  st.a = a;
  st.rs = load_res(p, seg);
  st.cl = clean_from(p, st.rs, a);
  st.general = (!st.rs.learning && st.rs.kind == 3 && !(a.smin >= a.smax && !a.nan)) ? 1 : 0;
  return st;
}

__device__ __forceinline__ int shfl_i(int v, int lane) { return __shfl(v, lane, 64); }
__device__ __forceinline__ double shfl_d(double v, int lane) { return shfl_any(v, lane); }

}  // namespace dm
