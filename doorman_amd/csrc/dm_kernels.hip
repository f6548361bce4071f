// dm_kernels.hip — gfx950 kernels for one apportionment tick.
//
// Every lease row is decided against the same frozen store (include/doorman_hip.h).
// Per resource the reference's per-request loops (go/server/doorman/algorithm.go)
// collapse to segmented reductions:
//   Clean          store.go:169-181   pass A: expired-row sums (parity) or live sums
//   ProportionalShare algorithm.go:213-293  pass B: extraCapacity / extraNeed, then map
//   FairShare      algorithm.go:95-206    pass B: extra / wantExtra (round 1),
//                                         pass C: extraExtra / wantExtraExtra at T (round 2), then map
//   NoAlgorithm / Static / Learn  algorithm.go:66-84,297-302  map only
// The path is HBM-bound (48 B per lease, ~15 flops): no MFMA.  Rows are read once
// from HBM into VGPRs and every pass runs from registers; the large-resource path
// re-reads from L2 / Infinity Cache.
//
// Float semantics follow Go on amd64: binary64, no FMA contraction (built with
// -ffp-contract=off), minF = `l > r ? r : l`, IEEE division by zero.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "dm_kernel_util.h"

namespace dm {

// --------------------------------------------------------------------------
// Resource-per-group kernel: G threads (a wave or a 256-thread workgroup) own
// one resource of up to G*R rows; rows live in VGPRs across all passes.
// --------------------------------------------------------------------------
// MODE (the 128/256/512-thread bins): kMixed = one kernel for every item (hint or
// not), kDenseOnly = items whose hint is set (k_block_dense: no subclients column at
// all; a stale hint queues the item for k_block_rest and returns), kRest = queued
// items (k_block_rest: the column is read, the hint rewritten).
enum { kMixed = 0, kDenseOnly = 1, kRest = 2 };
// Gets stores: non-temporal for the workgroup bins and the large chain (long contiguous
// spans: whole lines); plain for the sub-wave groups, whose spans are short and
// unaligned, so that L2 merges the partial sectors two groups write at a resource
// boundary (C2 112.2-112.5 -> 109.6-111.1 us, three interleaved rounds; the chain's
// stores plain: no change; profiles/r05_ab/c2_gets_stores.txt)
template <int G> constexpr bool kGroupNT = G >= 128;
constexpr bool kSpecNT = true;

template <int G, int R, int MODE = kMixed>
__device__ __forceinline__ void group_segment(const DevParams& p, const WorkItem wi, WorkItem* item, int t,
                                              Lds<G>& lds, int32_t* general_list, int32_t* general_count,
                                              int32_t* queue = nullptr, int32_t* qcount = nullptr,
                                              int32_t qidx = 0, int32_t* guard = nullptr, int qcap = 0) {
  // the dense state (below): every workgroup kernel tracks it and writes the hints;
  // only the 128-thread mixed kernel and the dense-only kernels load by the hint
  constexpr bool kDense = G >= 128 || (G == 64 && R >= 16);  // (64 x 16: kBin4Wave)
  constexpr bool kHintLoad = (G == 128 && MODE == kMixed) || MODE == kDenseOnly;
  const int seg = wi.seg;
  const int64_t lo = wi.lo;
  const int n = kDense ? wi.n & 0xFFFF : wi.n;
  // wave-uniform bases + 32-bit per-lane offsets: one VGPR addresses every column
  const double* __restrict__ wb = p.wants + lo;
  const double* __restrict__ hb = p.has + lo;
  const int32_t* __restrict__ sb = p.sub + lo;
  const int64_t* __restrict__ eb = p.expiry + lo;
  // the rows stay in VGPRs for every pass: 6 registers per row
  double w[R], h[R];
  int s[R];   // subclients in [0, kSubMax]
  int sr[R];  // the raw subclients words: where each row's expiry lives (dm_device.h)
  unsigned valid = 0, live = 0;
  unsigned relm = 0;  // rows a dense resource's mask says are released (bit k: row k*G + t)
  unsigned relb = 0;  // rows whose subclients word marks them released
  // Every load is issued before any is consumed: lanes past the segment end
  // re-read row n-1 (same cache line, n >= 1 in every bin) instead of branching
  // around the load, which made the compiler wait on each row's expiry before
  // issuing the next row (R serial memory latencies per workgroup).
  // A dense resource (every row a live follower with the same subclients s0, the
  // state its last writeback tick left: dm_device.h) is not read from the
  // subclients column: 24 B per lease instead of 28.  The work item carries the
  // state as a hint (no dependent load before the rows); the resource's own byte,
  // loaded with its record, confirms it, and a stale hint (an upsert or release
  // since that tick) reads the column after all.  The 128-thread mixed kernel
  // (257-1024 rows) loads by the hint; the 256/512-thread mixed kernels (1025-4096
  // rows) only track the state and write the hints (the extra branch costs
  // registers they do not have: spills at 5 waves per SIMD, C2 +3.5 %), and their
  // dense-only kernels skip the column.
  // A dense resource may also hold released rows (C2: loaded leases that had lapsed):
  // its hint word carries "has released rows" (bit 8) and the tick that set it wrote
  // which rows they are, one mask entry of R bits per lane (RelMask), read here in
  // place of the column: 1-2 B per lane instead of 4 B per row.
  const int hw = kDense ? wi.n >> 16 : 0;  // hint word: s0 in bits 0-7, released rows in bit 8, arrivals in bit 9
  const int hint = (kHintLoad) ? hw & 0xFF : 0;
  using MaskT = typename RelMask<R>::T;
  MaskT* const mrow = reinterpret_cast<MaskT*>(p.rmask + rel_mask_offset(lo));
  // rows upserted since the dense state was set (dm_device.h mask_pos): the high nibble
  // of the released-row entry for R <= 4, else G entries after the released-row ones
  constexpr unsigned kRowBits = R >= 32 ? ~0u : (1u << R) - 1u;
  const bool arrivals = kDense && ((hw >> 9) & 1);
  bool by_hint = MODE == kDenseOnly;  // the rows' states come from the hint and the masks, not the column
  if (MODE != kDenseOnly && !hint) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * G + t;
      const unsigned u = (unsigned)(i < n ? i : n - 1);
      // plain loads: non-temporal loads measured 3-4% slower (tools/ab.py, C1 and C3)
      w[k] = *col_at(wb, u);
      h[k] = *col_at(hb, u);
      sr[k] = *col_at(sb, u);
    }
  } else {
    if (hw >> 8 & 1) relm = (unsigned)mrow[t] & kRowBits;
    by_hint = true;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * G + t;
      const unsigned u = (unsigned)(i < n ? i : n - 1);
      w[k] = *col_at(wb, u);
      h[k] = *col_at(hb, u);
      sr[k] = hint;  // uniform: the mask's rows are taken out below (one register, not R)
    }
  }
  const Res rs = load_res(p, seg);
  // arrivals outlive the followers (at or after follow_exp): only a tick past follow_exp
  // needs their own expiries, from the columns
  const bool arr_lapse = arrivals && p.now > rs.follow_exp;
  if constexpr (MODE == kDenseOnly) {
    if (dense_subclients(rs) != hint || arr_lapse) {  // stale hint: k_block_rest reads the column
      if (t == 0) {
        const int q = atomicAdd(qcount, 1);
        if (q < qcap) queue[q] = qidx;  // at most one entry per item and tick (a guarded tick's count may grow)
        if (guard) __hip_atomic_store(guard, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return;
    }
  } else if (kHintLoad && hint && (dense_subclients(rs) != hint || arr_lapse)) {
    relm = 0;  // the column says which rows are released now
    by_hint = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * G + t;
      sr[k] = *col_at(sb, (unsigned)(i < n ? i : n - 1));
    }
  }
  // Followers expire with their resource; only a resource whose rows may carry an
  // explicit expiry (loaded / upserted by the host, none after a writeback tick)
  // reads the 8-B expiry column.  The test is the resource's flag, not the rows'
  // subclients words, which would make every wave wait for its loads to decide.
  int64_t e[R];
#pragma unroll
  for (int k = 0; k < R; ++k) e[k] = rs.follow_exp;
  if (MODE != kDenseOnly && (any_explicit(rs) || arr_lapse)) {  // a dense resource: only its lapsing arrivals
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = k * G + t;
      const int64_t x = *col_at(eb, (unsigned)(i < n ? i : n - 1));
      if (sub_explicit(sr[k])) e[k] = x;
    }
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {  // rows past the end stay out of valid/live, so every pass skips them
    const unsigned vk = (k * G + t < n) ? 1u : 0u;
    valid |= vk << k;
    if (sub_released(sr[k])) e[k] = kReleased;
    live |= (vk & (p.now > e[k] ? 0u : 1u)) << k;  // store.go:174 when.After(expiry)
    relb |= (sub_released(sr[k]) ? 1u : 0u) << k;
    s[k] = sub_value(sr[k]);
  }
  live &= ~relm;

  // ---- pass A: Clean ----
  AggA a = zeroA();
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (!(valid >> k & 1)) continue;
    const bool lv = live >> k & 1;
    const int sk = (relm >> k & 1) ? 0 : s[k];  // a released row counts nothing (its wants and has are 0)
    if (!lv) {
      a.cnt += sk;
      a.h += h[k];
      a.w += w[k];
    }
    if (p.recompute) {
      a.all.cnt += sk;
      a.all.h += h[k];
      a.all.w += w[k];
    }
    if (lv) {
      a.smin = s[k] < a.smin ? s[k] : a.smin;
      a.smax = s[k] > a.smax ? s[k] : a.smax;
      a.nan |= __builtin_isnan(w[k]) ? 1 : 0;
      a.nlive += 1;
    }
  }
  {
    const AggR all_part = a.all;
    bool fast_a = false;
    if constexpr (G <= 64) {
      // Sub-wave and wave groups are VALU-bound on their reductions.  In the steady
      // state pass A's totals are known wave-wide without one: no row of the wave is
      // released by this Clean (rows already marked released hold zeros), its live
      // rows share one subclient count u, no wants is NaN.  Then every group's Clean
      // sums are exact zeros and its live range is [u, u] (empty: no live row).
      if (!p.recompute) {
        const uint64_t lv = __ballot(live != 0);
        const int u = __builtin_amdgcn_readlane(a.smin, lv ? (int)__builtin_ctzll(lv) : 0);
        const bool ok = (valid & ~live & ~relb) == 0 && a.cnt == 0 && __double_as_longlong(a.h) == 0 &&
                        __double_as_longlong(a.w) == 0 && !a.nan && (live == 0 || (a.smin == u && a.smax == u));
        if (__all(ok)) {
          fast_a = true;
          const int base = (int)(threadIdx.x & 63) & ~(G - 1);
          uint64_t gmask = ~0ull;
          if constexpr (G < 64) gmask = ((1ull << G) - 1) << base;
          const bool any_live = (lv & gmask) != 0;
          a.smin = any_live ? u : INT32_MAX;
          a.smax = any_live ? u : INT32_MIN;
        }
      }
    }
    if (!fast_a) a = group_reduce<G, AggA, OpA, false>(a, OpA(), lds.a);
    if (p.recompute) a.all = group_reduce<G, AggR, OpR, false>(all_part, OpR(), lds.r);
  }
  const Clean cl = clean_from(p, rs, a);
  const double C = rs.C;
  const double eq = C / (double)cl.count;  // algorithm.go:123,229 equalShare
  const bool ps = !rs.learning && rs.kind == 2;
  const bool fs = !rs.learning && rs.kind == 3;
  const bool fs_uniform = fs && a.smin >= a.smax && !a.nan;  // no live rows counts as uniform
  if (fs && !fs_uniform) {
    // heterogeneous subclients (GetServerCapacity, server.go:850-879) or NaN wants:
    // one round-2 threshold per distinct subclient count.  Rare (the hierarchy's
    // root level), so the whole resource goes to k_general, untouched here.
    if (t == 0) {
      general_list[atomicAdd(general_count, 1)] = seg;
      if (p.writeback && (wi.n >> 16)) item->n = n;  // k_general's writeback clears the byte
    }
    return;
  }

  // ---- pass B: ProportionalShare extraCapacity/extraNeed, FairShare round 1 ----
  AggB b{0.0, 0.0, 0};
  if (ps || fs) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (!(live >> k & 1)) continue;
      if (ps) {
        const double e = eq * (double)s[k];  // :273
        if (w[k] < e)
          b.x += e - w[k];  // :275
        else
          b.y += w[k] - e;  // :277
      } else {
        const double d = (double)s[k] * eq;  // :160
        if (w[k] < d)
          b.x += d - w[k];  // :164
        else if (w[k] > d)
          b.i += s[k];  // :168
      }
    }
    b = group_reduce<G, AggB, OpB, false>(b, OpB(), lds.b);
  }

  // ---- pass C (uniform subclients): FairShare round 2 at the resource's one threshold ----
  AggC cu{0.0, 0};
  FsU fu{0.0, 0.0, 0.0, 0.0, 0.0};
  if (fs_uniform) {
    fu = make_fsu(eq, a.smin, b.x, b.i, cu);
    const double Tu = fu.T;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (!(live >> k & 1)) continue;
      if (!(w[k] > (double)s[k] * eq)) continue;  // j in wantExtraClients (:165-169)
      if (w[k] < Tu)
        cu.ee += Tu - w[k];  // :197-198
      else if (w[k] > Tu)
        cu.sgt += s[k];  // :199-200
    }
    cu = group_reduce<G, AggC, OpC, false>(cu, OpC(), lds.c);
    fu = make_fsu(eq, a.smin, b.x, b.i, cu);
    if constexpr (G >= 64) fu = uniform(fu);  // one resource per wave or workgroup: SGPRs
  }

  // ---- map: decide and write every lease (store.go:153-167 Assign) ----
  SumD delta{0.0};
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (!(valid >> k & 1)) continue;
    const unsigned u = (unsigned)(k * G + t);
    if (!(live >> k & 1)) {  // released by Clean: no lease
      put_released<kGroupNT<G>>(p, lo, u, (relm >> k & 1) ? (int)kSubReleased : sr[k]);
      continue;
    }
    double g;
    if (rs.learning) {
      g = h[k];  // Learn (algorithm.go:297-302)
    } else if (rs.kind == 0) {
      g = w[k];  // NoAlgorithm
    } else if (rs.kind == 1) {
      g = minF(C, w[k]);  // Static
    } else if (ps) {
      const double epc = eq * (double)s[k];         // :233
      const double unused = C - cl.sum_has + h[k];  // :239
      g = (cl.sum_wants <= C || w[k] <= epc) ? minF(w[k], unused)            // :245
                                             : minF(epc + (w[k] - epc) * (b.x / b.y), unused);  // :283
    } else {
      g = fs_uniform_row(w[k], h[k], C, cl.sum_has, fu);
    }
    put_live<kGroupNT<G>>(p, lo, u, g, rs, sr[k]);
    delta.v += g - h[k];
  }
  // (uniform) the live arrivals of a dense resource decided by the hint become followers:
  // their explicit subclients words are rewritten (the arrival mask is loaded only here,
  // so a store without arrivals carries no register for it)
  unsigned arrm = 0;
  if (arrivals && by_hint) {
    arrm = R <= 4 ? ((unsigned)mrow[t] >> 4) & kRowBits : (unsigned)mrow[G + t];
    if (p.writeback) {
#pragma unroll
      for (int k = 0; k < R; ++k)
        if ((arrm & live) >> k & 1) *col_at(p.out_sub + lo, (unsigned)(k * G + t)) = hint;
    }
  }

  // After a writeback tick every live row follows the resource and every other row
  // is released: live rows with one subclient count s0 (1..254) make the resource
  // dense.  Released rows among them go into its mask (written by the tick that sets
  // the state; a dense tick leaves the state as it found it or, when the followers
  // lapse together, ends it).
  // A resource with no live row left (its followers lapsed together) stays dense,
  // every row in its mask, so that a dense tick always leaves a dense resource dense
  // (the host's skip of the rest kernel rests on it: dm_runtime.cpp).
  const int nlive = a.nlive;
  const int s_keep = (hw & 0xFF) ? (hw & 0xFF) : 1;
  const int dn = !(kDense && p.writeback) ? 0
                 : nlive == 0              ? s_keep
                 : (a.smin == a.smax && a.smin >= 1 && a.smin <= 254) ? a.smin : 0;
  const int hw_next = dn ? (dn | (nlive < n ? 1 << 8 : 0)) : 0;
  delta = group_reduce<G, SumD, OpSumD, false>(delta, OpSumD(), lds.d);
  // A dense tick changes the mask only by a lapse; a writeback tick that changes the
  // state word writes it whole (a later release ORs its row in, so it must be valid
  // whenever the hint is set) and clears the arrivals it turned into followers.
  if (kDense && (MODE == kDenseOnly ? nlive == 0 || (p.writeback && hw != hw_next)
                                    : (hw_next >> 8) != 0 || (p.writeback && hw != hw_next))) {
    // (R <= 4: a non-writeback tick keeps the arrivals' nibble)
    mrow[t] = (MaskT)((valid & ~live) | (R <= 4 && !p.writeback ? arrm << 4 : 0u));
    if (R > 4 && arrivals && p.writeback) mrow[G + t] = 0;
  }
  if (t == 0) {
    write_resource(p, seg, rs, cl, delta.v, dn);
    if (p.writeback && hw != hw_next) item->n = n | hw_next << 16;
  }
}

// One G-thread workgroup per resource (G = 128..512, R = 4 or 8 rows per thread).
// 257-1024 rows run on 128 threads (2 waves) with 8 rows each, held to 5 waves per
// SIMD (<= 96 VGPRs): 5 x 4 SIMDs x 64 lanes x 8 rows = 10240 rows in flight per CU
// against 7168 for 256 threads x 4 rows at 7 waves per SIMD (65 VGPRs).  The tick is
// bound by bytes in flight: C3 560-590 -> 490-500 us, C1 61 -> 55 us
// (tools/ab.py, one box); 6 waves per SIMD spills (80 VGPRs + scratch: 2x slower).
// 1025-2048 / 2049-4096 rows likewise on 256 x 8 (5 waves) / 512 x 8 (106 VGPRs, 4
// waves) instead of 512 x 4 / 1024 x 4: C2's kernel time -5%, its tick -2%.
template <int G, int R>
__global__ __launch_bounds__(G, (G <= 256 && R == 8) ? 5 : 1) void k_block(DevParams p, WorkItem* __restrict__ items, int nitems,
                                             int32_t* general_list, int32_t* general_count) {
  __shared__ Lds<G> lds;
  if ((int)blockIdx.x >= nitems) return;
  group_segment<G, R>(p, items[blockIdx.x], items + blockIdx.x, threadIdx.x, lds, general_list, general_count);
}

// The workgroup bins split by the dense hint (launch_bin_dense / launch_bin_rest):
// k_block_dense decides the items whose hint is set without the subclients column
// (128 x 8: 70 VGPRs, 7 waves per SIMD instead of 5, 14336 rows in flight per CU)
// and queues the others; k_block_rest decides the queue with the mixed body, a grid
// striding over it (sized from the last split tick's queue; an empty queue costs
// one small launch).  qcnt is a two-slot ring: this tick's count in qcnt[par], and
// k_block_rest clears qcnt[par ^ 1] for the next tick (stream order); host_count
// (host-mapped) tells the host how many items went to the queue (its choice of
// split or mixed), written only when the count differs from the last one written
// (qcnt[2]): a system-scope store to host memory keeps an otherwise empty launch
// alive ~2 us longer, every tick of a dense store.
// When the host skips k_block_rest (every item of the bin verified dense in this row
// epoch, dm_runtime.cpp), `guard` (host-mapped) is set should the dense kernel queue
// an item after all, which the host reports as DM_E_INTERNAL (and refuses the store)
// instead of leaving the item undecided unnoticed.  The tick's last kernel (this one,
// or the rest kernel) is launched with the tick's stop event when another queue waits
// for the tick (dm_runtime.cpp tick_ev).
// (128 x 8 held to 7 waves per SIMD: 71 VGPRs + 20 B of spill, C3 430 -> 590 us; round 5.)
template <int G, int R>
__global__ __launch_bounds__(G) void k_block_dense(DevParams p, WorkItem* __restrict__ items, int nitems,
                                                   int32_t* queue, int32_t* qcnt, int par,
                                                   int32_t* general_list, int32_t* general_count,
                                                   int32_t* guard) {
  __shared__ Lds<G> lds;
  if ((int)blockIdx.x < nitems) {
    const WorkItem wi = items[blockIdx.x];
    if ((wi.n >> 16) == 0) {
      if (threadIdx.x == 0) {
        const int q = atomicAdd(qcnt + par, 1);
        if (q < nitems) queue[q] = (int32_t)blockIdx.x;
        if (guard) __hip_atomic_store(guard, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    } else {
      group_segment<G, R, kDenseOnly>(p, wi, items + blockIdx.x, threadIdx.x, lds, general_list, general_count,
                                      queue, qcnt + par, (int32_t)blockIdx.x, guard, nitems);
    }
  }
}

template <int G, int R>
__global__ __launch_bounds__(G) void k_block_rest(DevParams p, WorkItem* __restrict__ items,
                                                  const int32_t* __restrict__ queue, int32_t* qcnt, int par,
                                                  int32_t* host_count, int32_t* general_list, int32_t* general_count) {
  __shared__ Lds<G> lds;
  const int count = qcnt[par];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    qcnt[par ^ 1] = 0;
    if (host_count && qcnt[2] != count) {
      __hip_atomic_store(host_count, count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      qcnt[2] = count;
    }
  }
  for (int q = blockIdx.x; q < count; q += gridDim.x) {
    const int idx = queue[q];
    group_segment<G, R, kRest>(p, items[idx], items + idx, threadIdx.x, lds, general_list, general_count);
    __syncthreads();  // the next item reuses the single-use LDS slots
  }
}

// One workgroup: how many items of a workgroup bin are not dense after a writeback
// tick, published to host-mapped memory as {count, epoch} (count first, the epoch
// with release order) -- the host's once-per-epoch check before it skips the bin's
// k_block_rest (dm_runtime.cpp).
__global__ __launch_bounds__(1024) void k_count_undense(const WorkItem* __restrict__ items, int n,
                                                        unsigned long long* rec, unsigned long long epoch) {
  __shared__ int part[16];
  int c = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) c += (items[i].n >> 16) == 0 ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += part[w];
    __hip_atomic_store(rec, (unsigned long long)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(rec + 1, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Sub-wave groups: G = 8, 16 or 32 lanes own one resource of up to G*R rows (R rows
// per lane), so a wave decides 64 / G resources with one set of reduction chains
// (DPP inside each 16-lane row, plus one readlane combine for G = 32); G = 64 is one
// wave per resource (wave reductions only, no barriers).  Small resources are
// VALU-bound on their per-resource reductions (~28 reduced dwords per pass set, 4 DPP
// steps each): narrow groups with several rows per lane share every DPP step among
// 64 / G resources.
// The sub-wave bins in one launch (k_subs): the workgroups of each bin follow one
// another in blockIdx order, so the class stream runs them without a kernel boundary
// (drain + ramp) between bins.  Register use is the largest bin's.
template <int G, int R>
__device__ __forceinline__ void sub_part(const DevParams& p, WorkItem* __restrict__ items, int nitems, int blk,
                                         int32_t* general_list, int32_t* general_count) {
  Lds<G> lds;  // unused by sub-wave and wave reductions
  const int i = blk * (256 / G) + (int)(threadIdx.x / G);
  if (i >= nitems) return;
  group_segment<G, R>(p, items[i], items + i, threadIdx.x & (G - 1), lds, general_list, general_count);
}

template <int K>
__device__ __forceinline__ void sub_shape(const DevParams& p, const SubBins& sb, int b, int32_t* general_list,
                                          int32_t* general_count) {
  if constexpr (K < kSubShapes) {
    if (b < sb.blocks[K])
      return sub_part<kSubShapeG[K], kSubShapeR[K]>(p, sb.items[K], sb.n[K], b, general_list, general_count);
    sub_shape<K + 1>(p, sb, b - sb.blocks[K], general_list, general_count);
  }
}

__global__ __launch_bounds__(256, 5) void k_subs(DevParams p, SubBins sb, int32_t* general_list,
                                              int32_t* general_count) {
  sub_shape<0>(p, sb, (int)blockIdx.x, general_list, general_count);
}

// --------------------------------------------------------------------------
// Tiles of small resources (n <= kSmallMax), one 256-thread workgroup per tile
// (dm_device.h Tile): the workgroup stages the tile's rows in LDS with lane-strided
// (coalesced) loads while thread k loads resource k's offsets and record (consecutive
// records: coalesced as well) -- one memory round trip, where the packed kernel waits
// for its pack, then for the records its rows' resources name.  Thread k then decides
// resource k literally, in row order (sums in the oracle's order: bit-exact), from LDS;
// the gets go back to global memory row-parallel (coalesced), and each resource's
// record from its thread (coalesced).
// --------------------------------------------------------------------------
struct TileLds {
  double w[kTileRows];
  double h[kTileRows];  // a row's has, then its gets (only the row's own resource thread reads either)
  int32_t sr[kTileRows];
  uint8_t lv[kTileRows];
};

__global__ __launch_bounds__(256) void k_tile_small(DevParams p, const Tile* __restrict__ tiles,
                                                    const TileEntry* __restrict__ list) {
  __shared__ TileLds L;
  const Tile tl = tiles[blockIdx.x];
  const int t = threadIdx.x;
  const bool lst = tl.list != 0;  // (uniform)
  const int nrows = tl.nrows, nseg = tl.nseg;
  constexpr int K = kTileRows / 256;
  // the records first, then the rows: every load of the tile is in flight before the
  // first is consumed (the LDS stores below)
  const bool own = t < nseg;
  int seg, ldo = 0;
  if (lst) {
    const TileEntry e = list[tl.first_seg + (own ? t : 0)];
    seg = e.seg;
    ldo = e.lds;
  } else {
    seg = tl.first_seg + (own ? t : 0);
  }
  const int64_t lo64 = p.seg_off[seg], hi64 = p.seg_off[seg + 1];
  // a row's global index is base + its LDS index (a list tile: per resource)
  const int64_t row0 = lst ? lo64 - ldo : tl.row0;
  const Res rs = load_res(p, seg);
  if (lst) {  // each thread its own resource's rows (n <= kSmallMax)
    const int n = own ? (int)(hi64 - lo64) : 0;
    double wv[kSmallMax], hv[kSmallMax];
    int sv[kSmallMax];
#pragma unroll
    for (int j = 0; j < kSmallMax; ++j)
      if (j < n) {
        wv[j] = p.wants[lo64 + j];
        hv[j] = p.has[lo64 + j];
        sv[j] = p.sub[lo64 + j];
      }
#pragma unroll
    for (int j = 0; j < kSmallMax; ++j)
      if (j < n) {
        L.w[ldo + j] = wv[j];
        L.h[ldo + j] = hv[j];
        L.sr[ldo + j] = sv[j];
      }
  } else {
    double wv[K], hv[K];
    int sv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (k * 256 < nrows) {  // uniform
        const int i = k * 256 + t;
        const unsigned u = (unsigned)(i < nrows ? i : nrows - 1);
        wv[k] = *col_at(p.wants + row0, u);
        hv[k] = *col_at(p.has + row0, u);
        sv[k] = *col_at(p.sub + row0, u);
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = k * 256 + t;
      if (k * 256 < nrows && i < nrows) {
        L.w[i] = wv[k];
        L.h[i] = hv[k];
        L.sr[i] = sv[k];
      }
    }
  }
  __syncthreads();
  if (own) {
    const int lo = (int)(lo64 - row0), hi = (int)(hi64 - row0);
    // Clean (store.go:169-181): the store's running sums (or rebuilt from every row in
    // row order, recompute mode) less the rows that expired, in row order
    long long count;
    double sh, sw;
    if (p.recompute) {
      count = 0;
      sh = 0.0;
      sw = 0.0;
      for (int q = lo; q < hi; ++q) {
        sh += L.h[q] - 0.0;
        sw += L.w[q] - 0.0;
        count += sub_value(L.sr[q]);
      }
    } else {
      count = rs.agg_count;
      sh = rs.agg_has;
      sw = rs.agg_wants;
    }
    const bool expl_rows = any_explicit(rs);
    unsigned live = 0;  // bit q - lo (n <= kSmallMax)
    for (int q = lo; q < hi; ++q) {
      const int32_t raw = L.sr[q];
      int64_t e = rs.follow_exp;
      if (expl_rows && sub_explicit(raw)) e = p.expiry[row0 + q];
      if (sub_released(raw)) e = kReleased;
      const bool lv = !(p.now > e);  // store.go:174
      live |= (lv ? 1u : 0u) << (q - lo);
      if (!lv && !sub_released(raw)) {  // expired: Clean releases it (a released row holds zeros)
        sw -= L.w[q];
        sh -= L.h[q];
        count -= sub_value(raw);
      }
    }
    const double C = rs.C;
    const double eq = C / (double)count;
    const bool ps = !rs.learning && rs.kind == 2, fs = !rs.learning && rs.kind == 3;
    double x = 0.0, y = 0.0;
    long long wi = 0;
    if (ps || fs) {
      for (int q = lo; q < hi; ++q) {
        if (!(live >> (q - lo) & 1)) continue;
        const double wj = L.w[q];
        const int sj = sub_value(L.sr[q]);
        if (ps) {
          const double e2 = eq * (double)sj;  // algorithm.go:273
          if (wj < e2)
            x += e2 - wj;
          else
            y += wj - e2;
        } else {
          const double d = (double)sj * eq;  // algorithm.go:160
          if (wj < d)
            x += d - wj;
          else if (wj > d)
            wi += sj;
        }
      }
    }
    double osh = sh;  // Assign: sumHas += gets - has (store.go:156), row order
    double Tc = 0.0;  // round 2 at the last threshold asked for (uniform subclients: one per resource)
    AggC cc{0.0, 0};
    bool have_c = false;
    for (int q = lo; q < hi; ++q) {
      const bool lv = live >> (q - lo) & 1;
      L.lv[q] = lv ? 1 : 0;
      if (!p.writeback) __builtin_nontemporal_store(lv ? (int64_t)rs.exp_out : (int64_t)kReleased,
                                                    col_at(p.out_expiry + row0, (uint32_t)q));
      if (!lv) {
        L.h[q] = 0.0;
        continue;
      }
      const double w = L.w[q], h = L.h[q];
      const int s = sub_value(L.sr[q]);
      double g;
      if (rs.learning) {
        g = h;  // Learn (algorithm.go:297-302)
      } else if (rs.kind == 0) {
        g = w;  // NoAlgorithm
      } else if (rs.kind == 1) {
        g = minF(C, w);  // Static
      } else if (ps) {
        const double epc = eq * (double)s;  // :233
        const double unused = C - sh + h;   // :239
        g = (sw <= C || w <= epc) ? minF(w, unused) : minF(epc + (w - epc) * (x / y), unused);
      } else {
        double T = 0.0;
        if (!fs_stage01(w, h, s, C, sh, eq, x, wi, &g, &T)) {
          if (!have_c || __double_as_longlong(T) != __double_as_longlong(Tc)) {
            cc = AggC{0.0, 0};
            for (int j = lo; j < hi; ++j) {  // round 2 at this row's threshold (algorithm.go:189-204)
              if (!(live >> (j - lo) & 1)) continue;
              const double wj = L.w[j];
              const int sj = sub_value(L.sr[j]);
              if (!(wj > (double)sj * eq)) continue;
              if (wj < T)
                cc.ee += T - wj;
              else if (wj > T)
                cc.sgt += sj;
            }
            Tc = T;
            have_c = true;
          }
          g = fs_stage2(w, h, s, C, sh, eq, x, wi, T, cc);
        }
      }
      L.h[q] = g;
      osh += g - h;
    }
    write_resource(p, seg, rs, Clean{count, osh, sw}, 0.0);
  }
  if (lst) {  // a list tile: each thread its own resource's leases
    if (own) {
      for (int i = (int)(lo64 - row0); i < (int)(hi64 - row0); ++i) {
        const int32_t raw = L.sr[i];
        if (L.lv[i]) {
          __builtin_nontemporal_store(L.h[i], col_at(p.out_gets + row0, (uint32_t)i));
          if (p.writeback && raw < 0) *col_at(p.out_sub + row0, (uint32_t)i) = raw & 0x7FFFFFFF;
        } else {
          __builtin_nontemporal_store(0.0, col_at(p.out_gets + row0, (uint32_t)i));
          if (p.writeback && !sub_released(raw)) {
            *col_at(p.out_wants + row0, (uint32_t)i) = 0.0;
            *col_at(p.out_sub + row0, (uint32_t)i) = (int32_t)kSubReleased;
          }
        }
      }
    }
    return;
  }
  __syncthreads();
  // the leases, row-parallel (put_live / put_released of the packed kernel)
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = k * 256 + t;
    if (k * 256 < nrows && i < nrows) {
      const int32_t raw = L.sr[i];
      if (L.lv[i]) {
        __builtin_nontemporal_store(L.h[i], col_at(p.out_gets + row0, (uint32_t)i));
        if (p.writeback && raw < 0) *col_at(p.out_sub + row0, (uint32_t)i) = raw & 0x7FFFFFFF;
      } else {
        __builtin_nontemporal_store(0.0, col_at(p.out_gets + row0, (uint32_t)i));
        if (p.writeback && !sub_released(raw)) {
          *col_at(p.out_wants + row0, (uint32_t)i) = 0.0;
          *col_at(p.out_sub + row0, (uint32_t)i) = (int32_t)kSubReleased;
        }
      }
    }
  }
}

// --------------------------------------------------------------------------
// Large resources (n > kLargeMin): kChunkRows-row chunks, one workgroup each.
// Per-resource totals are re-derived in every workgroup from the chunk partials
// with the same fixed reduction tree, so all chunks of a resource agree exactly.
// --------------------------------------------------------------------------
struct SegTot {
  AggA a;
  AggB b;
  uint32_t pad[7];  // pad[0]: the map's arrival counter (k_large_map finishes the resource; its
                    // last arriver resets it)
  // nonzero when some chunk's Clean released subclients this tick (pass A, atomicOr),
  // i.e. round 1 must be recomputed; cleared by k_large_fin for the next tick.  With
  // it zero, pass B's other chunks return at once and its first chunk leaves the
  // speculative round-1 totals for C and the map (no O(chunks) re-reduction there)
  uint32_t rel;
};
static_assert(sizeof(SegTot) <= kSegTotBytes, "SegTot slot");
__device__ __forceinline__ SegTot* seg_tot(const Partials& P, int lseg) {
  return reinterpret_cast<SegTot*>(P.tot + (size_t)lseg * kSegTotBytes);
}

template <int G>
__device__ __forceinline__ SegState seg_state(const DevParams& p, const Partials& P, const LargeSeg& L,
                                              Lds<G>& lds) {
  AggA a = zeroA();
  for (int c = L.chunk_begin + (int)threadIdx.x; c < L.chunk_end; c += G) {
    AggA x;
    x.cnt = P.a_cnt[c];
    x.h = P.a_has[c];
    x.w = P.a_wants[c];
    x.all = AggR{P.a_cnt_all[c], P.a_has_all[c], P.a_wants_all[c]};
    x.smin = (int)P.a_smin[c];
    x.smax = (int)P.a_smax[c];
    x.nan = P.a_nan[c];
    x.nlive = 0;
    const AggR all = OpR()(a.all, x.all);  // OpA carries `all` through unchanged
    a = OpA()(a, x);
    a.all = all;
  }
  {
    const AggR all_part = a.all;
    a = group_reduce<G>(a, OpA(), lds.a);
    if (p.recompute) a.all = group_reduce<G>(all_part, OpR(), lds.r);
  }
  return seg_state_of(p, L.seg, a);
}

template <int G>
__device__ __forceinline__ AggB seg_b(const Partials& P, const LargeSeg& L, Lds<G>& lds) {
  AggB b{0.0, 0.0, 0};
  for (int c = L.chunk_begin + (int)threadIdx.x; c < L.chunk_end; c += G) b = OpB()(b, AggB{P.b_x[c], P.b_y[c], P.b_w[c]});
  return group_reduce<G>(b, OpB(), lds.b);
}

template <int G>
__device__ __forceinline__ AggC seg_c(const Partials& P, const LargeSeg& L, Lds<G>& lds) {
  AggC c{0.0, 0};
  for (int q = L.chunk_begin + (int)threadIdx.x; q < L.chunk_end; q += G) c = OpC()(c, AggC{P.c_ee[q], P.c_sgt[q]});
  return group_reduce<G>(c, OpC(), lds.c);
}

// kChunkRows rows of one chunk, kLR per thread, loaded in one batch (all loads in
// flight before the first use).
constexpr int kLR = kChunkRows / 256;
struct ChunkRows {
  double w[kLR], h[kLR];
  int s[kLR];
  unsigned valid, live;
  unsigned expl, rel;  // rows whose expiry is explicit / already marked released (dm_device.h)
};
// Pass A: wants and subclients of the chunk's rows (loads issued before any is
// consumed, see group_segment), liveness from the expiry encoding, then has for
// the rows Clean releases only (every row in recompute mode): the steady state
// reads 12 of a lease's 20 bytes here (C2: 122 -> 73 MB per tick).
// uni >= 0: the subclients words are not read -- a row whose bit in prev_live (the
// last writeback tick's live bits, Partials::s_live) is set holds uni, any other row is
// marked released
template <bool ALLH = false>  // ALLH: has of every row, loaded beside wants (the speculative chain)
__device__ __forceinline__ void load_chunk(const DevParams& p, const Chunk& ch, ChunkRows& r, const Res& rs,
                                           int uni = -1, uint32_t prev_live = 0) {
  const double* __restrict__ wb = p.wants + ch.row0;
  const double* __restrict__ hb = p.has + ch.row0;
  const int32_t* __restrict__ sb = p.sub + ch.row0;
  const int64_t* __restrict__ eb = p.expiry + ch.row0;
  r.valid = r.live = r.expl = r.rel = 0;
  int sr[kLR];
  // the wants loads leave first, whichever form follows: they wait only for the chunk
  // record, not for the per-chunk count (uni) that picks the form (one memory latency
  // less per workgroup in the steady state)
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    const int i = k * 256 + threadIdx.x;
    r.w[k] = wb[(unsigned)(i < ch.nrows ? i : ch.nrows - 1)];
    r.h[k] = ALLH ? hb[(unsigned)(i < ch.nrows ? i : ch.nrows - 1)] : 0.0;
  }
  if (uni >= 0) {
#pragma unroll
    for (int k = 0; k < kLR; ++k) sr[k] = (prev_live >> k & 1) ? uni : (int32_t)kSubReleased;
  } else {
#pragma unroll
    for (int k = 0; k < kLR; ++k) {
      const int i = k * 256 + threadIdx.x;
      sr[k] = sb[(unsigned)(i < ch.nrows ? i : ch.nrows - 1)];
    }
  }
  int64_t e[kLR];
#pragma unroll
  for (int k = 0; k < kLR; ++k) e[k] = rs.follow_exp;
  if (any_explicit(rs)) {  // the resource's flag (see group_segment)
#pragma unroll
    for (int k = 0; k < kLR; ++k) {
      const int i = k * 256 + threadIdx.x;
      const int64_t x = eb[(unsigned)(i < ch.nrows ? i : ch.nrows - 1)];
      if (sub_explicit(sr[k])) e[k] = x;
    }
  }
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    const unsigned vk = (k * 256 + (int)threadIdx.x < ch.nrows) ? 1u : 0u;
    r.valid |= vk << k;
    if (sub_released(sr[k])) e[k] = kReleased;
    r.live |= (vk & (p.now > e[k] ? 0u : 1u)) << k;
    r.expl |= (sub_explicit(sr[k]) ? 1u : 0u) << k;
    r.rel |= (sub_released(sr[k]) ? 1u : 0u) << k;
    r.s[k] = sub_value(sr[k]);
  }
  // a row already marked released holds has 0 (every path that marks one zeroes it)
  const unsigned need_h = ALLH ? 0u : p.recompute ? r.valid : (r.valid & ~r.live & ~r.rel);
  if (__any(need_h != 0)) {
#pragma unroll
    for (int k = 0; k < kLR; ++k)
      if (need_h >> k & 1) r.h[k] = hb[(unsigned)(k * 256 + threadIdx.x)];
  }
}

// Passes B, C and the map: wants (plus has / subclients where the pass uses them)
// of the chunk's rows and the live mask pass A left instead of re-reading expiry.
__device__ __forceinline__ void load_chunk_w(const DevParams& p, const Partials& P, const Chunk& ch,
                                             ChunkRows& r, bool with_sub, bool with_has = false) {
  const double* __restrict__ wb = p.wants + ch.row0;
  const double* __restrict__ hb = p.has + ch.row0;
  const int32_t* __restrict__ sb = p.sub + ch.row0;
  r.valid = 0;
  const uint32_t m = P.live[(size_t)blockIdx.x * 256 + threadIdx.x];
  r.live = m & 0xFFu;
  r.expl = (m >> 8) & 0xFFu;
  r.rel = (m >> 16) & 0xFFu;
  // every load issued before any is consumed (lanes past the chunk re-read its last
  // row, see group_segment): loads inside a per-lane branch made the compiler wait
  // for each row-block before issuing the next, eight memory latencies per chunk
  const int n = ch.nrows;
  int sr[kLR];
  // wants / has first, subclients after: with_sub comes from the resource's config
  // (ProportionalShare), which need not have arrived for the first loads to leave
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    const int i = k * 256 + threadIdx.x;
    const unsigned u = (unsigned)(i < n ? i : n - 1);
    r.w[k] = *col_at(wb, u);
    r.h[k] = with_has ? *col_at(hb, u) : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    const int i = k * 256 + threadIdx.x;
    sr[k] = with_sub ? *col_at(sb, (unsigned)(i < n ? i : n - 1)) : 0;
  }
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    const bool v = k * 256 + (int)threadIdx.x < n;
    r.valid |= (v ? 1u : 0u) << k;
    r.s[k] = v ? sub_value(sr[k]) : 0;
    if (!v) {
      r.w[k] = 0.0;
      r.h[k] = 0.0;
    }
  }
}

__device__ __forceinline__ HetRes* het_of(const Partials& P, int lseg) {
  return reinterpret_cast<HetRes*>(P.het + (size_t)lseg * sizeof(HetRes));
}
constexpr uint32_t kHetEmpty = 0xFFFFFFFFu;  // never a subclient count (<= kSubMax)

__device__ __forceinline__ bool het_insert(uint32_t* set, int* n, uint32_t key) {  // true when new
  uint32_t slot = (key * 0x9E3779B1u >> 23) & (2 * kHetMaxS - 1);
  for (int probe = 0; probe < 2 * kHetMaxS; ++probe, slot = (slot + 1) & (2 * kHetMaxS - 1)) {
    uint32_t cur = set[slot];
    if (cur == key) return false;
    if (cur == kHetEmpty) {
      cur = atomicCAS(&set[slot], kHetEmpty, key);
      if (cur == kHetEmpty) {
        atomicAdd(n, 1);
        return true;
      }
      if (cur == key) return false;
    }
  }
  atomicAdd(n, kHetMaxS + 1);  // table full: overflow
  return false;
}

// the same on the resource's set in global memory (agent-scope atomics; the
// chunks of a resource insert concurrently)
__device__ __forceinline__ void het_insert_global(uint32_t* set, int32_t* n, uint32_t key) {
  uint32_t slot = (key * 0x9E3779B1u >> 23) & (2 * kHetMaxS - 1);
  for (int probe = 0; probe < 2 * kHetMaxS; ++probe, slot = (slot + 1) & (2 * kHetMaxS - 1)) {
    uint32_t cur = __hip_atomic_load((gu32*)(set + slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return;
    if (cur == kHetEmpty) {
      cur = atomicCAS(set + slot, kHetEmpty, key);
      if (cur == kHetEmpty) {
        atomicAdd(n, 1);
        return;
      }
      if (cur == key) return;
    }
  }
  atomicAdd(n, kHetMaxS + 1);  // table full: overflow
}

// pass A (k_large_a, when P.s_set): the chunk's distinct subclient counts of live
// rows into its resource's set -- one insert for a chunk whose live rows share one
// count, else the chunk's own LDS set first, one global insert per distinct count
__device__ void chunk_s_insert(const Partials& P, int lseg, const ChunkRows& rw, const AggA& a) {
  __shared__ uint32_t set[2 * kHetMaxS];
  __shared__ int n;
  const int t = threadIdx.x;
  uint32_t* gset = P.s_set + (size_t)lseg * 2 * kHetMaxS;
  int32_t* gn = P.s_n + lseg;
  if (a.smin > a.smax) return;  // no live rows
  if (a.smin == a.smax) {
    if (t == 0) het_insert_global(gset, gn, (uint32_t)a.smin);
    return;
  }
  for (int i = t; i < 2 * kHetMaxS; i += 256) set[i] = kHetEmpty;
  if (t == 0) n = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kLR; ++k)
    if (rw.live >> k & 1) het_insert(set, &n, (uint32_t)rw.s[k]);
  __syncthreads();
  if (n > kHetMaxS) {
    if (t == 0) atomicAdd(gn, kHetMaxS + 1);
    return;
  }
  for (int i = t; i < 2 * kHetMaxS; i += 256)
    if (set[i] != kHetEmpty) het_insert_global(gset, gn, set[i]);
}

__global__ __launch_bounds__(256) void k_large_a(DevParams p, const Chunk* __restrict__ chunks, Partials P) {
  __shared__ Lds<256> lds;
  const Chunk ch = chunks[blockIdx.x];
  const Res rs = load_res(p, ch.seg);
  ChunkRows rw;
  {
    const int uni = P.s_live ? __builtin_amdgcn_readfirstlane(P.uni[blockIdx.x]) : -1;
    const uint32_t prev_live = P.s_live ? P.live[(size_t)blockIdx.x * 256 + threadIdx.x] : 0u;
    load_chunk(p, ch, rw, rs, uni, prev_live);
  }
  AggA a = zeroA();
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.valid >> k & 1)) continue;
    const bool lv = rw.live >> k & 1;
    if (!lv) {
      a.cnt += rw.s[k];
      a.h += rw.h[k];
      a.w += rw.w[k];
    }
    if (p.recompute) {
      a.all.cnt += rw.s[k];
      a.all.h += rw.h[k];
      a.all.w += rw.w[k];
    }
    if (lv) {
      a.smin = rw.s[k] < a.smin ? rw.s[k] : a.smin;
      a.smax = rw.s[k] > a.smax ? rw.s[k] : a.smax;
      a.nan |= __builtin_isnan(rw.w[k]) ? 1 : 0;
    }
  }
  P.live[(size_t)blockIdx.x * 256 + threadIdx.x] = rw.live | rw.expl << 8 | rw.rel << 16;
  // Speculative pass B (ProportionalShare / FairShare outside learning mode) with
  // equalShare from the store's running Count.  It is exactly pass B's result
  // whenever Clean releases no subclients of the resource (same eq, same live
  // rows, same per-chunk summation order); k_large_b checks that and recomputes
  // otherwise.  Saves pass B's row reads (12 B per lease) in the steady state.
  const bool spec = !p.recompute && !rs.learning && rs.kind >= 2;
  AggB b{0.0, 0.0, 0};
  if (spec) {
    const double eq = rs.C / (double)rs.agg_count;
#pragma unroll
    for (int k = 0; k < kLR; ++k) {
      if (!(rw.live >> k & 1)) continue;
      const double w = rw.w[k];
      const int sk = rw.s[k];
      if (rs.kind == 2) {
        const double e = eq * (double)sk;  // algorithm.go:273
        if (w < e)
          b.x += e - w;
        else
          b.y += w - e;
      } else {
        const double d = (double)sk * eq;  // algorithm.go:160
        if (w < d)
          b.x += d - w;
        else if (w > d)
          b.i += sk;
      }
    }
  }
  {
    const AggR all_part = a.all;
    if (P.s_set)  // every thread reads the chunk's count range (chunk_s_insert)
      a = group_reduce<256>(a, OpA(), lds.a);
    else
      a = group_reduce_t0<256>(a, OpA(), lds.a);
    if (p.recompute) a.all = group_reduce_t0<256>(all_part, OpR(), lds.r);
    if (spec) b = group_reduce_t0<256>(b, OpB(), lds.b);
  }
  if (P.s_set && !rs.learning && rs.kind == 3) chunk_s_insert(P, ch.lseg, rw, a);  // heterogeneous FairShare
  if (threadIdx.x == 0) {
    const int c = blockIdx.x;
    if (a.cnt != 0) atomicOr(&seg_tot(P, ch.lseg)->rel, 1u);
    if (spec) {
      P.b_x[c] = b.x;
      P.b_y[c] = b.y;
      P.b_w[c] = b.i;
    }
    P.a_cnt[c] = a.cnt;
    P.a_cnt_all[c] = a.all.cnt;
    P.a_has_all[c] = a.all.h;
    P.a_wants_all[c] = a.all.w;
    P.a_has[c] = a.h;
    P.a_wants[c] = a.w;
    P.a_smin[c] = a.smin;
    P.a_smax[c] = a.smax;
    P.a_nan[c] = a.nan;
  }
}

__global__ __launch_bounds__(256) void k_large_b(DevParams p, const Chunk* __restrict__ chunks,
                                                 const LargeSeg* __restrict__ ls, Partials P) {
  __shared__ Lds<256> lds;
  // P.b_first: one workgroup per large resource, as its first chunk (pass A's
  // speculative round 1 is exact: the store holds no explicit-expiry rows, so Clean
  // releases none of the resource's live rows or all of them, and then round 1 sums
  // nothing either way)
  const int ci = P.b_first ? ls[blockIdx.x].chunk_begin : (int)blockIdx.x;
  const Chunk ch = chunks[ci];
  // most chunks leave here: their resource's round 1 is exact from pass A and they
  // are not its first chunk (no config load on that path)
  const LargeSeg L = ls[ch.lseg];
  const bool first = ci == L.chunk_begin;
  const bool spec_ok = P.b_first || (!p.recompute && seg_tot(P, ch.lseg)->rel == 0);  // pass A's partials are exact
  if (spec_ok && !first) return;
  bool ps;
  {  // only ProportionalShare / FairShare outside learning mode need this pass
    const ResCfg cf = p.cfg[ch.seg];
    if (cf.learning_end_ns > p.now || cf.kind < 2) return;
    ps = cf.kind == 2;
  }
  const SegState st = seg_state<256>(p, P, L, lds);
  if (threadIdx.x == 0 && first) seg_tot(P, ch.lseg)->a = st.a;
  const bool het = st.general && P.s_set;  // heterogeneous FairShare decided on the chain
  if ((st.general && !het) || st.rs.learning || st.rs.kind < 2) return;
  if (spec_ok) {  // the first chunk leaves the speculative round-1 totals (C and the map read them)
    const AggB b = seg_b<256>(P, L, lds);
    if (threadIdx.x == 0) seg_tot(P, ch.lseg)->b = b;
    return;
  }
  ChunkRows rw;
  load_chunk_w(p, P, ch, rw, ps || het);
  const double eq = st.rs.C / (double)st.cl.count;
  if (!ps && !het) {  // uniform FairShare: one count
#pragma unroll
    for (int k = 0; k < kLR; ++k) rw.s[k] = st.a.smin;
  }
  AggB b{0.0, 0.0, 0};
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.live >> k & 1)) continue;
    const double w = rw.w[k];
    const int s = rw.s[k];
    if (st.rs.kind == 2) {
      const double e = eq * (double)s;
      if (w < e)
        b.x += e - w;
      else
        b.y += w - e;
    } else {
      const double d = (double)s * eq;
      if (w < d)
        b.x += d - w;
      else if (w > d)
        b.i += s;
    }
  }
  b = group_reduce_t0<256>(b, OpB(), lds.b);
  if (threadIdx.x == 0) {
    P.b_x[blockIdx.x] = b.x;
    P.b_y[blockIdx.x] = b.y;
    P.b_w[blockIdx.x] = b.i;
  }
}

__global__ __launch_bounds__(256) void k_large_c(DevParams p, const Chunk* __restrict__ chunks,
                                                 const LargeSeg* __restrict__ ls, Partials P) {
  __shared__ Lds<256> lds;
  const Chunk ch = chunks[blockIdx.x];
  {  // only FairShare outside learning mode has a round 2
    const ResCfg cf = p.cfg[ch.seg];
    if (cf.learning_end_ns > p.now || cf.kind != 3) return;
  }
  ChunkRows rw;
  load_chunk_w(p, P, ch, rw, false);  // rows in flight while the resource's partials are reduced
  const LargeSeg L = ls[ch.lseg];
  const SegState st = seg_state_of(p, L.seg, seg_tot(P, ch.lseg)->a);  // left by pass B
  if (st.general || st.rs.learning || st.rs.kind != 3) return;
#pragma unroll
  for (int k = 0; k < kLR; ++k) rw.s[k] = st.a.smin;  // uniform subclients here
  const bool spec_ok = !p.recompute && seg_tot(P, ch.lseg)->rel == 0;  // pass B's first chunk left b
  const AggB b = spec_ok ? seg_tot(P, ch.lseg)->b : seg_b<256>(P, L, lds);
  if (threadIdx.x == 0 && !spec_ok && (int)blockIdx.x == L.chunk_begin) seg_tot(P, ch.lseg)->b = b;
  const double eq = st.rs.C / (double)st.cl.count;
  const double s0 = (double)st.a.smin;
  const double Tu = (b.x / (double)b.i) * s0 + eq * s0;
  AggC c{0.0, 0};
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.live >> k & 1)) continue;
    const double w = rw.w[k];
    const int s = rw.s[k];
    if (!(w > (double)s * eq)) continue;
    if (w < Tu)
      c.ee += Tu - w;
    else if (w > Tu)
      c.sgt += s;
  }
  c = group_reduce_t0<256>(c, OpC(), lds.c);
  if (threadIdx.x == 0) {
    P.c_ee[blockIdx.x] = c.ee;
    P.c_sgt[blockIdx.x] = c.sgt;
  }
}

// The map of one chunk (store.go:153-167 Assign): decide and write every lease of its
// rows under the resource's totals; returns the chunk's sum of gets - has.  (k_large_map
// keeps its own copy of the loop: called, that kernel spilled 68 B per lane.)
__device__ __forceinline__ double map_chunk(const DevParams& p, const Chunk& ch, const ChunkRows& rw, const Res rs,
                                            const Clean cl, const AggB b, const FsU fu) {
  const double C = rs.C;
  const double eq = C / (double)cl.count;
  double delta = 0.0;
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.valid >> k & 1)) continue;
    const unsigned u = (unsigned)(k * 256 + threadIdx.x);
    const double w = rw.w[k], h = rw.h[k];
    if (!(rw.live >> k & 1)) {  // released by Clean (the raw word for put_released: marked or not)
      put_released(p, ch.row0, u, (rw.rel >> k & 1) ? (int32_t)kSubReleased : 0);
      continue;
    }
    double g;
    if (rs.learning) {
      g = h;
    } else if (rs.kind == 0) {
      g = w;
    } else if (rs.kind == 1) {
      g = minF(C, w);
    } else if (rs.kind == 2) {
      const double epc = eq * (double)rw.s[k];
      const double unused = C - cl.sum_has + h;
      g = (cl.sum_wants <= C || w <= epc) ? minF(w, unused) : minF(epc + (w - epc) * (b.x / b.y), unused);
    } else {
      g = fs_uniform_row(w, h, C, cl.sum_has, fu);
    }
    // an explicit row becomes a follower (its subclients word without the flag)
    put_live(p, ch.row0, u, g, rs, (rw.expl >> k & 1) ? (p.sub[ch.row0 + u] | (int32_t)kSubExplicit) : 0);
    delta += g - h;
  }
  return delta;
}

__global__ __launch_bounds__(256) void k_large_map(DevParams p, const Chunk* __restrict__ chunks,
                                                   const LargeSeg* __restrict__ ls, Partials P, int32_t* glist,
                                                   int32_t* gcount) {
  __shared__ Lds<256> lds;
  const Chunk ch = chunks[blockIdx.x];
  bool ps, fs;
  {
    const ResCfg cf = p.cfg[ch.seg];
    const bool lrn = cf.learning_end_ns > p.now;
    ps = !lrn && cf.kind == 2;
    fs = !lrn && cf.kind == 3;
  }
  ChunkRows rw;
  load_chunk_w(p, P, ch, rw, ps, true);  // rows in flight while the resource's partials are reduced
  const LargeSeg L = ls[ch.lseg];
  // pass A totals: left by pass B for ProportionalShare / FairShare
  const SegState st =
      uniform((ps || fs) ? seg_state_of(p, L.seg, seg_tot(P, ch.lseg)->a) : seg_state<256>(p, P, L, lds));
  // Without the heterogeneous chain (P.s_set) the map also does k_large_fin's work: the
  // resource's last-arriving chunk sums the chunks' deltas and writes its record
  const bool finish = P.s_set == nullptr;
  if (st.general) {  // k_general decides it; its first chunk lists it (fin's job)
    if (threadIdx.x == 0) P.uni[blockIdx.x] = -1;
    if (finish && threadIdx.x == 0 && (int)blockIdx.x == L.chunk_begin) {
      glist[atomicAdd(gcount, 1)] = L.seg;
      seg_tot(P, ch.lseg)->rel = 0;
    }
    return;
  }
  const Res& rs = st.rs;
  const double C = rs.C;
  const double eq = C / (double)st.cl.count;
  AggB b{0.0, 0.0, 0};
  AggC c{0.0, 0};
  if (ps) b = (!p.recompute && seg_tot(P, ch.lseg)->rel == 0) ? seg_tot(P, ch.lseg)->b : seg_b<256>(P, L, lds);
  if (fs) {
    b = seg_tot(P, ch.lseg)->b;  // left by pass C
    c = seg_c<256>(P, L, lds);
  }
  b = uniform(b);  // the resource's totals stay in SGPRs through the map
  const FsU fu = uniform(make_fsu(eq, st.a.smin, b.x, b.i, c));  // SGPRs through the map
  SumD delta{0.0};
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.valid >> k & 1)) continue;
    const unsigned u = (unsigned)(k * 256 + threadIdx.x);
    const double w = rw.w[k], h = rw.h[k];
    if (!(rw.live >> k & 1)) {  // released by Clean (the raw word for put_released: marked or not)
      put_released(p, ch.row0, u, (rw.rel >> k & 1) ? (int32_t)kSubReleased : 0);
      continue;
    }
    double g;
    if (rs.learning) {
      g = h;
    } else if (rs.kind == 0) {
      g = w;
    } else if (rs.kind == 1) {
      g = minF(C, w);
    } else if (rs.kind == 2) {
      const double epc = eq * (double)rw.s[k];
      const double unused = C - st.cl.sum_has + h;
      g = (st.cl.sum_wants <= C || w <= epc) ? minF(w, unused) : minF(epc + (w - epc) * (b.x / b.y), unused);
    } else {
      g = fs_uniform_row(w, h, C, st.cl.sum_has, fu);
    }
    // an explicit row becomes a follower (its subclients word without the flag)
    put_live(p, ch.row0, u, g, rs, (rw.expl >> k & 1) ? (p.sub[ch.row0 + u] | (int32_t)kSubExplicit) : 0);
    delta.v += g - h;
  }
  delta = group_reduce_t0<256>(delta, OpSumD(), lds.d);
  if (threadIdx.x == 0)  // after a writeback tick every row this left live holds it (Partials::s_live)
    P.uni[blockIdx.x] = st.a.smin == st.a.smax ? st.a.smin : -1;
  if (!finish) {
    if (threadIdx.x == 0) P.d_delta[blockIdx.x] = delta.v;
    return;
  }
  if (threadIdx.x >= 64) return;  // wave 0 hands off (dm_kernel_util.h: write-through, then arrive)
  if (threadIdx.x == 0) st_wt(P.d_delta + blockIdx.x, delta.v);
  SegTot* tt = seg_tot(P, ch.lseg);
  if (!arrive_last(&tt->pad[0], L.chunk_end - L.chunk_begin)) return;
  SumD d{0.0};
  for (int q = L.chunk_begin + (int)threadIdx.x; q < L.chunk_end; q += 64) d.v += ld_wt(P.d_delta + q);
  d = wave_reduce(d, OpSumD());
  if (threadIdx.x == 0) {
    tt->rel = 0;  // pass A of the next tick sets it again (every chunk has read it)
    write_resource(p, L.seg, rs, st.cl, d.v);
  }
}

// --------------------------------------------------------------------------
// The speculative chain (the steady state of P.b_first ticks, DM_SPEC_CHAIN).
// k_large_spec: one launch over every chunk.  Each chunk computes its exact pass-A
// partials and its round-1 partials (equalShare from the running Count, as pass A's
// speculative round 1), its round-2 partials at the threshold the resource's stored
// totals give (SpecTot: its last tick's), and writes its leases under those stored
// totals -- unless its own rows show a lapse, a NaN wants or another count, when it
// writes nothing.  The resource's last-arriving chunk (no waiting) reduces the
// partials with one fixed tree and compares them bit for bit with the stored totals:
// equal, the leases written are exactly the chain's (the same totals, the same rows)
// and it writes the resource's record; else it marks the resource for
// k_large_redo.  Per lease: wants and has read, gets written -- one pass instead of
// the chain's four launches and second read.
// k_large_redo_team: one launch, every workgroup leaves at once when nothing is
// marked.  A marked resource's chunks are shared by a team of at most kTeamMax
// workgroups that meet twice at most (round 1 again when Clean released rows, round
// 2), through write-through partials, the last arriver's write-through total and a
// ready flag (the launch number); they then rewrite their leases and the last arriver
// stores the totals as the next tick's speculation.  Only a team waits for itself, so
// any grid of >= kTeamMax co-resident workgroups finishes; a wait is still bounded
// (kSpecSpin polls: the host then reports DM_E_INTERNAL and refuses the store until it
// is reloaded).
// --------------------------------------------------------------------------
constexpr uint32_t kSpecSpin = 1u << 22;  // polls of ~0.1 us

__device__ __forceinline__ bool dbl_pos0(double x) { return __double_as_longlong(x) == 0; }

// wave 0's fixed reduction over a resource's chunk partials (lane l: chunks begin + l,
// begin + l + 64, ... in order, then the wave's DPP tree); every lane gets the total
template <typename T, typename Op, typename Ld>
__device__ __forceinline__ T canon_reduce(int begin, int end, T v, Op op, Ld ld) {
  for (int q = begin + (int)(threadIdx.x & 63); q < end; q += 64) v = op(v, ld(q));
  return wave_reduce(v, op);
}
__device__ __forceinline__ AggA canon_a(const Partials& P, const LargeSeg& L) {
  return canon_reduce(L.chunk_begin, L.chunk_end, zeroA(), OpA(), [&](int q) {
    AggA x = zeroA();
    x.cnt = ld_wt(P.a_cnt + q);
    x.h = ld_wt(P.a_has + q);
    x.w = ld_wt(P.a_wants + q);
    x.smin = (int)ld_wt(P.a_smin + q);
    x.smax = (int)ld_wt(P.a_smax + q);
    x.nan = ld_wt(P.a_nan + q);
    return x;
  });
}
__device__ __forceinline__ AggB canon_b(const Partials& P, const LargeSeg& L) {
  return canon_reduce(L.chunk_begin, L.chunk_end, AggB{0.0, 0.0, 0}, OpB(),
                      [&](int q) { return AggB{ld_wt(P.b_x + q), ld_wt(P.b_y + q), ld_wt(P.b_w + q)}; });
}
__device__ __forceinline__ AggC canon_c(const Partials& P, const LargeSeg& L) {
  return canon_reduce(L.chunk_begin, L.chunk_end, AggC{0.0, 0}, OpC(),
                      [&](int q) { return AggC{ld_wt(P.c_ee + q), ld_wt(P.c_sgt + q)}; });
}
__device__ __forceinline__ double canon_d(const Partials& P, const LargeSeg& L) {
  return canon_reduce(L.chunk_begin, L.chunk_end, SumD{0.0}, OpSumD(),
                      [&](int q) { return SumD{ld_wt(P.d_delta + q)}; }).v;
}
// canon_a, canon_b, canon_c and canon_d in one pass over the chunks (k_large_spec's
// verifier): every partial of a 64-chunk stripe loaded at once, one round trip per
// stripe instead of four; each quantity keeps its own order and tree (the same bits)
struct CanonAll {
  AggA a;
  AggB b;
  AggC c;
  double d;
};
__device__ __forceinline__ CanonAll canon_all(const Partials& P, const LargeSeg& L) {
  AggA a = zeroA();
  AggB b{0.0, 0.0, 0};
  AggC c{0.0, 0};
  SumD d{0.0};
  for (int q = L.chunk_begin + (int)(threadIdx.x & 63); q < L.chunk_end; q += 64) {
    AggA x = zeroA();
    x.cnt = ld_wt(P.a_cnt + q);
    x.h = ld_wt(P.a_has + q);
    x.w = ld_wt(P.a_wants + q);
    x.smin = (int)ld_wt(P.a_smin + q);
    x.smax = (int)ld_wt(P.a_smax + q);
    x.nan = ld_wt(P.a_nan + q);
    const AggB y{ld_wt(P.b_x + q), ld_wt(P.b_y + q), ld_wt(P.b_w + q)};
    const AggC z{ld_wt(P.c_ee + q), ld_wt(P.c_sgt + q)};
    const SumD u{ld_wt(P.d_delta + q)};
    a = OpA()(a, x);
    b = OpB()(b, y);
    c = OpC()(c, z);
    d = OpSumD()(d, u);
  }
  return CanonAll{wave_reduce(a, OpA()), wave_reduce(b, OpB()), wave_reduce(c, OpC()), wave_reduce(d, OpSumD()).v};
}

// pass A (Clean sums of the rows it releases, the live rows' count range, NaN wants)
// and round 1 with equalShare eq over the chunk's rows in registers (as k_large_a)
__device__ __forceinline__ AggA chunk_a(const ChunkRows& rw) {
  AggA a = zeroA();
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.valid >> k & 1)) continue;
    if (!(rw.live >> k & 1)) {
      a.cnt += rw.s[k];
      a.h += rw.h[k];
      a.w += rw.w[k];
    } else {
      a.smin = rw.s[k] < a.smin ? rw.s[k] : a.smin;
      a.smax = rw.s[k] > a.smax ? rw.s[k] : a.smax;
      a.nan |= __builtin_isnan(rw.w[k]) ? 1 : 0;
    }
  }
  return a;
}
__device__ __forceinline__ AggB chunk_b(const ChunkRows& rw, int kind, double eq) {
  AggB b{0.0, 0.0, 0};
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.live >> k & 1)) continue;
    const double w = rw.w[k];
    const int sk = rw.s[k];
    if (kind == 2) {
      const double e = eq * (double)sk;  // algorithm.go:273
      if (w < e)
        b.x += e - w;
      else
        b.y += w - e;
    } else {
      const double d = (double)sk * eq;  // algorithm.go:160
      if (w < d)
        b.x += d - w;
      else if (w > d)
        b.i += sk;
    }
  }
  return b;
}
// round 2 at threshold Tu over the live rows, every one holding s0 (k_large_c)
__device__ __forceinline__ AggC chunk_c(const ChunkRows& rw, int s0, double eq, double Tu) {
  AggC x{0.0, 0};
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.live >> k & 1)) continue;
    const double w = rw.w[k];
    if (!(w > (double)s0 * eq)) continue;
    if (w < Tu)
      x.ee += Tu - w;
    else if (w > Tu)
      x.sgt += s0;
  }
  return x;
}

// (at 5 waves per SIMD -- amdgpu_waves_per_eu(5): 96 VGPRs, 2 spilled -- C2 lost 105.2 ->
// 108.7 us, both orders, round 6: the chain's workgroups are latency-bound per phase,
// and the spill sits on the map's path)
__global__ __launch_bounds__(256) void k_large_spec(DevParams p, const Chunk* __restrict__ chunks,
                                                    const LargeSeg* __restrict__ ls, Partials P, SpecArgs S) {
  __shared__ Lds<256> lds;
  __shared__ int s_ok;
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  const Chunk ch = chunks[c];
  const Res rs = load_res(p, ch.seg);
  SpecTot* sp = S.tot + ch.lseg;
  ChunkRows rw;
  {
    const int uni = P.s_live ? __builtin_amdgcn_readfirstlane(P.uni[c]) : -1;
    const uint32_t prev_live = P.s_live ? P.live[(size_t)c * 256 + t] : 0u;
    load_chunk<true>(p, ch, rw, rs, uni, prev_live);
  }
  const int valid = sp->valid, s0 = sp->s0;  // the stored totals (written by earlier launches)
  const AggB bs{sp->bx, sp->by, sp->bi};
  const AggC cs{sp->cee, sp->csgt};
  AggA a = chunk_a(rw);
  P.live[(size_t)c * 256 + t] = rw.live | rw.expl << 8 | rw.rel << 16;
  const bool r1 = !rs.learning && rs.kind >= 2;
  const bool fs = !rs.learning && rs.kind == 3;
  const double eq = rs.C / (double)rs.agg_count;  // the running Count: exact when Clean releases nothing
  AggB b = r1 ? chunk_b(rw, rs.kind, eq) : AggB{0.0, 0.0, 0};
  a = group_reduce_t0<256>(a, OpA(), lds.a);
  if (r1) b = group_reduce_t0<256>(b, OpB(), lds.b);
  if (t == 0)  // this chunk's rows agree with the speculation: nothing released, one count s0, no NaN
    s_ok = (valid && a.cnt == 0 && dbl_pos0(a.h) && dbl_pos0(a.w) && !a.nan &&
            (a.smin > a.smax || (a.smin == s0 && a.smax == s0)))
               ? 1
               : 0;
  __syncthreads();
  const bool ok = s_ok != 0;
  AggC x{0.0, 0};
  SumD delta{0.0};
  if (ok) {
    AggA z = zeroA();
    z.smin = z.smax = s0;
    const Clean cl = clean_from(p, rs, z);  // the running sums: the Clean of a tick that releases nothing
    const FsU fu = uniform(make_fsu(eq, s0, bs.x, bs.i, cs));
    if (fs) x = group_reduce_t0<256>(chunk_c(rw, s0, eq, fu.T), OpC(), lds.c);
    delta.v = map_chunk(p, ch, rw, rs, cl, uniform(bs), fu);
    delta = group_reduce_t0<256>(delta, OpSumD(), lds.d);
  }
  if (t == 0) {
    st_wt(P.a_cnt + c, (int64_t)a.cnt);
    st_wt(P.a_has + c, a.h);
    st_wt(P.a_wants + c, a.w);
    st_wt(P.a_smin + c, (int64_t)a.smin);
    st_wt(P.a_smax + c, (int64_t)a.smax);
    st_wt(P.a_nan + c, a.nan);
    st_wt(P.b_x + c, b.x);
    st_wt(P.b_y + c, b.y);
    st_wt(P.b_w + c, (int64_t)b.i);
    st_wt(P.c_ee + c, x.ee);
    st_wt(P.c_sgt + c, (int64_t)x.sgt);
    st_wt(P.d_delta + c, delta.v);
    P.uni[c] = ok ? s0 : -1;  // the redo rewrites a marked resource's
    if (!ok) __hip_atomic_store((gu32*)&sp->redo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t >= 64) return;  // wave 0 verifies (dm_kernel_util.h arrive_last)
  const LargeSeg L = ls[ch.lseg];
  if (!arrive_last(&sp->arrive[0], L.chunk_end - L.chunk_begin)) return;
  const CanonAll ca = canon_all(P, L);
  const AggA at = ca.a;
  const AggB bt = ca.b;
  const AggC ct = ca.c;
  const bool marked = __hip_atomic_load((gu32*)&sp->redo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  bool same = valid && !marked && at.cnt == 0 && dbl_pos0(at.h) && dbl_pos0(at.w) && !at.nan &&
              (at.smin > at.smax || (at.smin == s0 && at.smax == s0));
  if (rs.kind == 2 && !rs.learning)
    same = same && __double_as_longlong(bt.x) == __double_as_longlong(bs.x) &&
           __double_as_longlong(bt.y) == __double_as_longlong(bs.y);
  if (fs)
    same = same && __double_as_longlong(bt.x) == __double_as_longlong(bs.x) && bt.i == bs.i &&
           __double_as_longlong(ct.ee) == __double_as_longlong(cs.ee) && ct.sgt == cs.sgt;
  if (same) {
    const double d = ca.d;
    if (t == 0) {
      AggA z = zeroA();
      z.smin = z.smax = s0;
      write_resource(p, L.seg, rs, clean_from(p, rs, z), d);
    }
    return;
  }
  if (t == 0) {  // the redo's inputs: the actual pass-A totals and round 1 at the running Count
    sp->redo = 1;
    S.ring[S.par] = 1;  // (read by the next launch)
    sp->a_cnt = at.cnt;
    sp->a_h = at.h;
    sp->a_w = at.w;
    sp->a_smin = at.smin;
    sp->a_smax = at.smax;
    sp->a_nan = at.nan;
    sp->abx = bt.x;
    sp->aby = bt.y;
    sp->abi = bt.i;
  }
}

// every thread's write-through stores have landed, then one arrival; true (uniform)
// for the last arriver, which resets the counter
__device__ __forceinline__ bool spec_arrive(uint32_t* ctr, int nch, int* s_last) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add((gu32*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (uint32_t)nch - 1 ? 1 : 0;
    if (last) __hip_atomic_store((gu32*)ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = last;
  }
  __syncthreads();
  return *s_last != 0;
}
__device__ __forceinline__ void spec_ready(const SpecArgs& S, uint64_t* flag) {  // the last arriver's stores landed
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_wt(flag, S.seq + 1);
  }
}
__device__ __forceinline__ void spec_wait(const SpecArgs& S, const uint64_t* flag) {
  if (threadIdx.x == 0) {
    for (uint32_t it = 0; ld_wt(flag) < S.seq + 1; ++it) {
      if (it >= kSpecSpin) {
        __hip_atomic_store(S.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __syncthreads();
}

// The redo by teams: a marked resource's chunks are shared among W = min(chunks,
// kTeamMax) workgroups (its team slots, in ticket order), each taking every W-th chunk
// through each phase, its rows loaded again per phase.  Every chunk partial is one
// 256-thread reduction and every total one canonical tree (canon_*), so the bits are
// those the chain would write; only a team waits for itself, so any grid of >= kTeamMax
// co-resident workgroups finishes (no bound on a resource's chunks).  (Round 4's
// per-chunk redo, one workgroup per chunk with every chunk of a resource co-resident,
// was retired in round 5.)
// Two builds of the same code: the full one and a light one held to 64 VGPRs (8 waves;
// a chunk's rows spill to scratch).  A steady tick marks nothing, and there the launch
// is all the redo costs: the light build's workgroups find a free slot beside the
// other classes' waves much sooner (C2: 20 -> 10 us of event time, the tick -3.6 us),
// while a redo of every large resource takes it about 2x as long.  The host launches
// the light build while the last redo it saw found nothing marked and no row changed
// since (dm_runtime.cpp); both leave the same bits.
__device__ __forceinline__ void redo_team(const DevParams& p, const Chunk* __restrict__ chunks,
                                          const LargeSeg* __restrict__ ls, const Partials& P, const SpecArgs& S,
                                          int32_t* glist, int32_t* gcount, int l, int m, Lds<256>& lds,
                                          int* s_last_p) {
  int& s_last = *s_last_p;
  const int t = threadIdx.x;
  SpecTot* sp = S.tot + l;
  const LargeSeg L = ls[l];
  const int nch = L.chunk_end - L.chunk_begin;
  const int W = nch < kTeamMax ? nch : kTeamMax;
  AggA at = zeroA();
  at.cnt = sp->a_cnt;
  at.h = sp->a_h;
  at.w = sp->a_w;
  at.smin = sp->a_smin;
  at.smax = sp->a_smax;
  at.nan = sp->a_nan;
  const SegState st = uniform(seg_state_of(p, L.seg, at));
  const Res rs = st.rs;
  if (st.general) {  // k_general decides it (its member 0 lists it)
    for (int c = L.chunk_begin + m; c < L.chunk_end; c += W)
      if (t == 0) P.uni[c] = -1;
    if (t == 0 && m == 0) {
      glist[atomicAdd(gcount, 1)] = L.seg;
      sp->redo = 0;
      sp->valid = 0;
    }
    return;
  }
  const bool r1 = !rs.learning && rs.kind >= 2;
  const bool fs = !rs.learning && rs.kind == 3;
  const double eq = rs.C / (double)st.cl.count;
  AggB bt{sp->abx, sp->aby, sp->abi};  // round 1 at the running Count: exact when Clean released nothing
  if (r1 && at.cnt != 0) {  // round 1 again at the Count after Clean
    for (int c = L.chunk_begin + m; c < L.chunk_end; c += W) {
      ChunkRows rw;
      load_chunk<true>(p, chunks[c], rw, rs);
      const AggB x = group_reduce_t0<256>(chunk_b(rw, rs.kind, eq), OpB(), lds.b);
      if (t == 0) {
        st_wt(P.b_x + c, x.x);
        st_wt(P.b_y + c, x.y);
        st_wt(P.b_w + c, (int64_t)x.i);
      }
      __syncthreads();
    }
    if (spec_arrive(&sp->arrive[1], W, &s_last)) {
      if (t < 64) {
        const AggB r = canon_b(P, L);
        if (t == 0) {
          st_wt(&sp->abx, r.x);
          st_wt(&sp->aby, r.y);
          st_wt(reinterpret_cast<int64_t*>(&sp->abi), (int64_t)r.i);
        }
      }
      spec_ready(S, &sp->ready[0]);
    }
    spec_wait(S, &sp->ready[0]);
    bt = AggB{ld_wt(&sp->abx), ld_wt(&sp->aby), ld_wt(reinterpret_cast<const int64_t*>(&sp->abi))};
  }
  const int s0 = st.a.smin;
  AggC ct{0.0, 0};
  FsU fu = make_fsu(eq, s0, bt.x, bt.i, ct);
  if (fs) {  // round 2 at the resource's threshold
    for (int c = L.chunk_begin + m; c < L.chunk_end; c += W) {
      ChunkRows rw;
      load_chunk<true>(p, chunks[c], rw, rs);
      const AggC x = group_reduce_t0<256>(chunk_c(rw, s0, eq, fu.T), OpC(), lds.c);
      if (t == 0) {
        st_wt(P.c_ee + c, x.ee);
        st_wt(P.c_sgt + c, (int64_t)x.sgt);
      }
      __syncthreads();
    }
    if (spec_arrive(&sp->arrive[2], W, &s_last)) {
      if (t < 64) {
        const AggC r = canon_c(P, L);
        if (t == 0) {
          st_wt(&sp->cee, r.ee);
          st_wt(reinterpret_cast<int64_t*>(&sp->csgt), (int64_t)r.sgt);
        }
      }
      spec_ready(S, &sp->ready[1]);
    }
    spec_wait(S, &sp->ready[1]);
    ct = AggC{ld_wt(&sp->cee), ld_wt(reinterpret_cast<const int64_t*>(&sp->csgt))};
    fu = make_fsu(eq, s0, bt.x, bt.i, ct);
  }
  for (int c = L.chunk_begin + m; c < L.chunk_end; c += W) {
    ChunkRows rw;
    const Chunk ch = chunks[c];
    load_chunk<true>(p, ch, rw, rs);
    SumD delta{map_chunk(p, ch, rw, rs, st.cl, uniform(bt), uniform(fu))};
    delta = group_reduce_t0<256>(delta, OpSumD(), lds.d);
    if (t == 0) {
      P.uni[c] = st.a.smin == st.a.smax ? st.a.smin : -1;
      st_wt(P.d_delta + c, delta.v);
    }
    __syncthreads();
  }
  if (!spec_arrive(&sp->arrive[0], W, &s_last)) return;
  if (t >= 64) return;
  const double d = canon_d(P, L);
  if (t == 0) {
    write_resource(p, L.seg, rs, st.cl, d);
    // the next tick's speculation: this tick's totals (round 1 and 2 as the chunks used
    // them; a resource whose live rows hold mixed counts is not speculated on)
    sp->bx = bt.x;
    sp->by = bt.y;
    sp->bi = bt.i;
    sp->cee = ct.ee;
    sp->csgt = ct.sgt;
    sp->s0 = s0;
    sp->valid = (st.a.smin >= st.a.smax) ? 1 : 0;  // one count, or no live row
    sp->redo = 0;
  }
}

// Team slots in ticket order (a resource's slots consecutive): with a grid of >=
// kTeamMax workgroups only the team at the ticket front can have members not yet taken
template <bool kLight>
__global__ __launch_bounds__(256, kLight ? 8 : 1) void k_large_redo_team(DevParams p, const Chunk* __restrict__ chunks,
                                                                          const LargeSeg* __restrict__ ls, Partials P,
                                                                          SpecArgs S, int32_t* glist, int32_t* gcount) {
  __shared__ Lds<256> lds;
  __shared__ int s_last, s_c;
  const int q = S.par ^ 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the next tick's slots (its k_large_spec runs after this)
    S.ring[q] = 0;
    S.ring[2 + q] = 0;
    // tell the host only that a redo ran (it clears the word when it reads it): a
    // system-scope store to host memory keeps an otherwise empty launch alive ~2 us
    // longer, and the steady tick's empty redo is on the large chain's critical path
    const uint32_t marked = S.ring[S.par];
    if (marked) __hip_atomic_store(S.seen, marked, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (!S.ring[S.par]) return;  // nothing marked (k_large_spec: the previous launch)
  for (;;) {
    if (threadIdx.x == 0) s_c = (int)atomicAdd(S.ring + 2 + S.par, 1u);
    __syncthreads();
    const int k = s_c;
    if (k >= S.nslots) return;
    const int32_t tm = S.team[k];
    const int l = tm >> 8, m = tm & 0xFF;
    if (S.tot[l].redo) redo_team(p, chunks, ls, P, S, glist, gcount, l, m, lds, &s_last);
    __syncthreads();  // every wave back before the next ticket
  }
}

__global__ __launch_bounds__(256) void k_large_fin(DevParams p, const LargeSeg* __restrict__ ls, Partials P,
                                                   int32_t* general_list, int32_t* general_count) {
  __shared__ Lds<256> lds;
  const LargeSeg L = ls[blockIdx.x];
  if (threadIdx.x == 0) seg_tot(P, blockIdx.x)->rel = 0;  // pass A of the next tick sets it again
  const SegState st = seg_state<256>(p, P, L, lds);
  if (st.general) {
    if (!P.s_set) {  // no heterogeneous path on the chain this tick: k_general decides it
      if (threadIdx.x == 0) general_list[atomicAdd(general_count, 1)] = L.seg;
      return;
    }
    if (het_of(P, blockIdx.x)->mode != 1) return;  // k_large_t handed it to k_general
  }
  SumD d{0.0};
  for (int c = L.chunk_begin + (int)threadIdx.x; c < L.chunk_end; c += 256) d.v += P.d_delta[c];
  d = group_reduce<256>(d, OpSumD(), lds.d);
  if (threadIdx.x == 0) write_resource(p, L.seg, st.rs, st.cl, d.v);
}

// --------------------------------------------------------------------------
// General FairShare: resources with heterogeneous subclients or NaN wants, from
// any size bin (appended to the worklist by the other kernels, which leave such
// a resource untouched); only the hierarchy's root level (GetServerCapacity)
// produces them.  One workgroup per resource: Clean, round 1, then round 2
// (algorithm.go:188-204), where every row has its own threshold
// T(s) = deservedExtra + deservedShare -- one value per distinct subclient count.
// Round 2 by sorted thresholds: the distinct finite thresholds T_1 < ... < T_K are
// collected in LDS (hash set, then a bitonic sort); one pass puts every
// wantExtra client's wants into one of 2K+1 buckets (between / equal to the
// thresholds, binary search) with per-bucket (count, sum of wants, sum of
// subclients) accumulated per wave in a fixed order (each 64-row tile sorted by
// bucket, segmented sums, one writer per bucket); prefix sums over the buckets
// then give every threshold's
//   extraExtra     = k(T)*T - sum(w_j < T)   (the algebraic form of
//                                             sum(T - w_j), within the tolerance)
//   wantExtraExtra = sum(s_j : w_j > T)
// in O(n log K) instead of one pass over the resource per threshold.  More than
// kGenMaxT thresholds, or a non-finite one, keep the per-threshold passes.
constexpr int kGenMaxT = 256;
constexpr int kGenBuckets = 2 * kGenMaxT + 1;
constexpr uint64_t kGenEmpty = ~0ull;  // a NaN pattern: never a finite threshold's bits
struct GenLds {
  uint64_t set[2 * kGenMaxT];  // threshold bit patterns, open addressing
  double T[kGenMaxT];          // sorted distinct thresholds
  double ee[kGenMaxT];         // extraExtra per threshold
  long long sgt[kGenMaxT];     // wantExtraExtra - own subclients, per threshold
  double accw[4][kGenBuckets];
  long long accs[4][kGenBuckets];
  int accc[4][kGenBuckets];
  int nT, overflow;
};

// ascending bitonic sort of one key per lane across the wave
__device__ __forceinline__ uint32_t wave_sort64(uint32_t key) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t other = (uint32_t)__shfl_xor((int)key, j, 64);
      const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
      key = keep_min ? (key < other ? key : other) : (key > other ? key : other);
    }
  }
  return key;
}

// m = number of thresholds below w; bucket 2m (strictly between) or 2m+1 (== T_m+1)
__device__ __forceinline__ int gen_bucket(const double* T, int K, double w) {
  int lo = 0, hi = K;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (T[mid] < w)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < K && T[lo] == w) ? 2 * lo + 1 : 2 * lo;
}

__device__ __forceinline__ int gen_index(const double* T, int K, double t) {  // T[k] == t
  int lo = 0, hi = K;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (T[mid] < t)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_general(DevParams p, const int32_t* __restrict__ list,
                                                 const int32_t* __restrict__ count) {
  __shared__ Lds<256> lds;
  __shared__ GenLds gs;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int nlist = *count;
  for (int idx = blockIdx.x; idx < nlist; idx += gridDim.x) {
    const int seg = list[idx];
    const int64_t lo = p.seg_off[seg], hi = p.seg_off[seg + 1];
    const Res rs = load_res(p, seg);
    // liveness and subclients from the expiry encoding (dm_device.h); explicit rows
    // keep their flag until the last pass, so every pass sees the same live set
    auto dead = [&](int64_t row) { return p.now > row_expiry(p, row, p.sub[row], rs.follow_exp); };
    auto sub_at = [&](int64_t row) -> long long { return sub_value(p.sub[row]); };
    AggA a = zeroA();
    for (int64_t row = lo + t; row < hi; row += 256) {
      const double w = p.wants[row], h = p.has[row];
      const long long s = sub_at(row);
      const bool lv = !(dead(row));
      if (!lv) {
        a.cnt += s;
        a.h += h;
        a.w += w;
      }
      if (p.recompute) {
        a.all.cnt += s;
        a.all.h += h;
        a.all.w += w;
      }
    }
    {
      const AggR all_part = a.all;
      a = group_reduce<256>(a, OpA(), lds.a);
      if (p.recompute) a.all = group_reduce<256>(all_part, OpR(), lds.r);
    }
    const Clean cl = clean_from(p, rs, a);
    const double C = rs.C;
    const double eq = C / (double)cl.count;
    // round 1 sums (algorithm.go:156-171)
    AggB b{0.0, 0.0, 0};
    for (int64_t row = lo + t; row < hi; row += 256) {
      if (dead(row)) continue;
      const double w = p.wants[row];
      const long long s = sub_at(row);
      const double d = (double)s * eq;
      if (w < d)
        b.x += d - w;
      else if (w > d)
        b.i += s;
    }
    b = group_reduce<256>(b, OpB(), lds.b);
    for (int i = t; i < 2 * kGenMaxT; i += 256) gs.set[i] = kGenEmpty;
    if (t == 0) {
      gs.nT = 0;
      gs.overflow = 0;
    }
    __syncthreads();
    // rows decided in round 0/1, released rows, NaN thresholds; the other rows'
    // thresholds into the set
    SumD delta{0.0};
    for (int64_t row = lo + t; row < hi; row += 256) {
      const double w = p.wants[row], h = p.has[row];
      const long long s = sub_at(row);
      if (dead(row)) {
        put_released(p, row, 0u, p.sub[row]);
        continue;
      }
      double g, T = 0.0;
      bool done = fs_stage01(w, h, s, C, cl.sum_has, eq, b.x, b.i, &g, &T);
      if (!done && __builtin_isnan(T)) {
        g = fs_stage2(w, h, s, C, cl.sum_has, eq, b.x, b.i, T, AggC{0.0, 0});
        done = true;
      }
      if (done) {
        __builtin_nontemporal_store(g, p.out_gets + row);
        if (!p.writeback) __builtin_nontemporal_store((int64_t)(rs.exp_out), p.out_expiry + row);
        delta.v += g - h;
      } else if (!__builtin_isfinite(T)) {
        gs.overflow = 1;  // +-Inf threshold: the per-threshold passes below
      } else {
        const uint64_t key = __builtin_bit_cast(uint64_t, T);
        uint32_t slot = (uint32_t)((key ^ (key >> 29)) * 0x9E3779B97F4A7C15ull >> 40) & (2 * kGenMaxT - 1);
        for (int probe = 0; probe < 2 * kGenMaxT; ++probe, slot = (slot + 1) & (2 * kGenMaxT - 1)) {
          uint64_t cur = gs.set[slot];
          if (cur == key) break;
          if (cur == kGenEmpty) {
            cur = atomicCAS((unsigned long long*)&gs.set[slot], (unsigned long long)kGenEmpty, (unsigned long long)key);
            if (cur == kGenEmpty) {
              if (atomicAdd(&gs.nT, 1) >= kGenMaxT) gs.overflow = 1;
              break;
            }
            if (cur == key) break;
          }
        }
      }
    }
    __syncthreads();
    const bool buckets = !gs.overflow;
    const int K = gs.nT;
    if (buckets && K > 0) {
      // the distinct thresholds, sorted: compact the set, pad with +Inf, bitonic sort
      __shared__ int nfill;
      if (t == 0) nfill = 0;
      __syncthreads();
      for (int i = t; i < 2 * kGenMaxT; i += 256)
        if (gs.set[i] != kGenEmpty) gs.T[atomicAdd(&nfill, 1)] = __builtin_bit_cast(double, gs.set[i]);
      __syncthreads();
      if (t >= K) gs.T[t] = __builtin_inf();
      for (int k = 2; k <= kGenMaxT; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
          __syncthreads();
          const int q = t ^ j;
          if (q > t) {
            const double x = gs.T[t], y = gs.T[q];
            const bool asc = (t & k) == 0;
            if ((x > y) == asc) {
              gs.T[t] = y;
              gs.T[q] = x;
            }
          }
        }
      for (int i = t; i < 4 * kGenBuckets; i += 256) {
        (&gs.accw[0][0])[i] = 0.0;
        (&gs.accs[0][0])[i] = 0;
        (&gs.accc[0][0])[i] = 0;
      }
      __syncthreads();
      // bucket pass over the wantExtra clients (w > d, algorithm.go:165-169): wave wv
      // takes 64-row tiles wv, wv+4, ... in order; in a tile the lanes are sorted by
      // bucket and each bucket's run summed in lane order
      for (int64_t base = lo + (int64_t)wv * 64; base < hi; base += 256) {
        const int64_t row = base + lane;
        double w = 0.0;
        long long s = 0;
        uint32_t bk = 0xFFFFu;
        if (row < hi && !(dead(row))) {
          w = p.wants[row];
          s = sub_at(row);
          if (w > (double)s * eq) bk = (uint32_t)gen_bucket(gs.T, K, w);
        }
        const uint32_t key = wave_sort64(bk << 6 | (uint32_t)lane);
        const int src = (int)(key & 63);
        const int mb = (int)(key >> 6);
        double vw = shfl_d(w, src);
        long long vs = __shfl(s, src, 64);
        int vc = mb != 0xFFFF ? 1 : 0;
        const int prevb = __shfl_up(mb, 1, 64);
        int run = (lane == 0 || prevb != mb) ? 1 : 0;  // first lane of its bucket's run
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {  // segmented inclusive scan, earlier + later
          const double ow = shfl_d(vw, lane >= off ? lane - off : lane);
          const long long os = __shfl(vs, lane >= off ? lane - off : lane, 64);
          const int oc = __shfl(vc, lane >= off ? lane - off : lane, 64);
          const int orun = __shfl(run, lane >= off ? lane - off : lane, 64);
          if (lane >= off && !run) {
            vw = ow + vw;
            vs = os + vs;
            vc = oc + vc;
            run = orun;
          }
        }
        const int nextb = __shfl_down(mb, 1, 64);
        if (mb != 0xFFFF && (lane == 63 || nextb != mb)) {  // last lane of its run: one writer per bucket
          gs.accw[wv][mb] += vw;
          gs.accs[wv][mb] += vs;
          gs.accc[wv][mb] += vc;
        }
      }
      __syncthreads();
      if (t == 0) {  // prefix over the buckets, waves combined in a fixed order
        long long cnt = 0, stot = 0;
        double sw = 0.0;
        for (int bb = 0; bb < 2 * K + 1; ++bb)
          stot += gs.accs[0][bb] + gs.accs[1][bb] + gs.accs[2][bb] + gs.accs[3][bb];
        long long sle = 0;  // subclients of buckets <= 2k-1 (w <= T_k)
        for (int k = 0; k < K; ++k) {
          // buckets 2k (below T_k) join the "below" sums; 2k+1 is w == T_k
          const int bl = 2 * k;
          cnt += gs.accc[0][bl] + gs.accc[1][bl] + gs.accc[2][bl] + gs.accc[3][bl];
          sw = sw + gs.accw[0][bl] + gs.accw[1][bl] + gs.accw[2][bl] + gs.accw[3][bl];
          sle += gs.accs[0][bl] + gs.accs[1][bl] + gs.accs[2][bl] + gs.accs[3][bl];
          const long long seq = gs.accs[0][bl + 1] + gs.accs[1][bl + 1] + gs.accs[2][bl + 1] + gs.accs[3][bl + 1];
          gs.ee[k] = cnt == 0 ? 0.0 : (double)cnt * gs.T[k] - sw;  // :197-198
          gs.sgt[k] = stot - sle - seq;                              // :199-200
          sle += seq;
          cnt += gs.accc[0][bl + 1] + gs.accc[1][bl + 1] + gs.accc[2][bl + 1] + gs.accc[3][bl + 1];
          sw = sw + gs.accw[0][bl + 1] + gs.accw[1][bl + 1] + gs.accw[2][bl + 1] + gs.accw[3][bl + 1];
        }
      }
      __syncthreads();
      for (int64_t row = lo + t; row < hi; row += 256) {
        if (dead(row)) continue;
        const double w = p.wants[row], h = p.has[row];
        const long long s = sub_at(row);
        double g, T = 0.0;
        if (fs_stage01(w, h, s, C, cl.sum_has, eq, b.x, b.i, &g, &T)) continue;
        if (__builtin_isnan(T)) continue;  // decided above
        const int k = gen_index(gs.T, K, T);
        g = fs_stage2(w, h, s, C, cl.sum_has, eq, b.x, b.i, T, AggC{gs.ee[k], gs.sgt[k]});
        __builtin_nontemporal_store(g, p.out_gets + row);
        if (!p.writeback) __builtin_nontemporal_store((int64_t)(rs.exp_out), p.out_expiry + row);
        delta.v += g - h;
      }
    } else if (!buckets) {
      // round 2 one distinct threshold at a time.  The rows written above keep
      // their inputs in registers only within their own pass, so round 2 re-reads
      // has from a resource that is already partly written back: only rows that are
      // still undecided are read, and those are untouched.
      double prev = 0.0;
      int have_prev = 0;
      for (;;) {
        TMin tm{0.0, 0, 0};
        for (int64_t row = lo + t; row < hi; row += 256) {
          if (dead(row)) continue;
          double g, T = 0.0;
          if (fs_stage01(p.wants[row], p.has[row], sub_at(row), C, cl.sum_has, eq, b.x, b.i, &g, &T)) continue;
          if (__builtin_isnan(T) || (have_prev && !(T > prev))) continue;
          tmin_add(tm, T);
        }
        tm = group_reduce<256>(tm, OpTMin(), lds.t);
        if (!tm.found) break;
        const double Ts = tm.t;
        AggC c{0.0, 0};
        for (int64_t row = lo + t; row < hi; row += 256) {
          if (dead(row)) continue;
          const double w = p.wants[row];
          const long long s = sub_at(row);
          if (!(w > (double)s * eq)) continue;
          if (w < Ts)
            c.ee += Ts - w;
          else if (w > Ts)
            c.sgt += s;
        }
        c = group_reduce<256>(c, OpC(), lds.c);
        for (int64_t row = lo + t; row < hi; row += 256) {
          if (dead(row)) continue;
          const double w = p.wants[row], h = p.has[row];
          const long long s = sub_at(row);
          double g, T = 0.0;
          if (fs_stage01(w, h, s, C, cl.sum_has, eq, b.x, b.i, &g, &T)) continue;
          if (!(T == Ts)) continue;
          g = fs_stage2(w, h, s, C, cl.sum_has, eq, b.x, b.i, T, c);
          __builtin_nontemporal_store(g, p.out_gets + row);
          if (!p.writeback) __builtin_nontemporal_store((int64_t)(rs.exp_out), p.out_expiry + row);
          delta.v += g - h;
        }
        prev = Ts;
        have_prev = 1;
      }
    }
    if (p.writeback) {  // every live explicit row becomes a follower of the resource's new expiry
      __syncthreads();
      for (int64_t row = lo + t; row < hi; row += 256) {
        const int32_t raw = p.sub[row];
        if (sub_explicit(raw) && !(p.now > p.expiry[row])) p.out_sub[row] = raw & 0x7FFFFFFF;
      }
    }
    delta = group_reduce<256>(delta, OpSumD(), lds.d);
    if (t == 0) write_resource(p, seg, rs, cl, delta.v);
    __syncthreads();  // the next resource reuses the LDS
  }
}


// --------------------------------------------------------------------------
// Heterogeneous-subclient FairShare of large resources on the chain (instead of
// one workgroup per resource in k_general): launched only when the store may hold
// such resources.  After pass B (round 1 with each row's own count):
//   k_large_t      per resource: round-1 totals, the distinct subclient counts of
//                  the live rows (from pass A's per-chunk lists) and their round-2
//                  thresholds T(s) = (E / W) s + eq s -- a row reaching round 2 has
//                  w > deservedShare, so its wantExtra is W and its threshold
//                  depends on its count only (algorithm.go:148,175,197) -- sorted;
//   k_large_c_het  per chunk: (count, sum wants, sum subclients) of the wantExtra
//                  clients per bucket between / at the thresholds (as k_general);
//   k_large_e      per resource: the chunks' buckets in chunk order, prefix sums:
//                  extraExtra(T) = k T - sum(w < T), wantExtraExtra(T) = sum(s : w > T);
//   k_large_map_het per chunk: every row decided (fs_stage01 / fs_stage2).
// More than kHetMaxS counts or a non-finite threshold: k_general (HetRes.mode 2).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_large_t(DevParams p, const LargeSeg* __restrict__ ls, Partials P,
                                                 int32_t* general_list, int32_t* general_count) {
  __shared__ Lds<256> lds;
  __shared__ uint32_t set[2 * kHetMaxS];
  __shared__ double T[kHetMaxS];
  __shared__ int n, fill;
  const int t = threadIdx.x;
  const LargeSeg L = ls[blockIdx.x];
  SegTot* tot = seg_tot(P, blockIdx.x);
  HetRes* H = het_of(P, blockIdx.x);
  uint32_t* gset = P.s_set + (size_t)blockIdx.x * 2 * kHetMaxS;
  // the resource's distinct counts (pass A), and the set emptied for the next tick
  for (int i = t; i < 2 * kHetMaxS; i += 256) {
    set[i] = gset[i];
    gset[i] = kHetEmpty;
  }
  if (t == 0) {
    n = P.s_n[blockIdx.x];
    P.s_n[blockIdx.x] = 0;
    fill = 0;
  }
  __syncthreads();
  const SegState st = seg_state_of(p, L.seg, tot->a);  // left by pass B's first chunk
  if (!st.general) {
    if (t == 0) H->mode = 0;
    return;
  }
  const AggB b = seg_b<256>(P, L, lds);  // round 1 with every row's own count: E = b.x, W = b.i
  if (t == 0) tot->b = b;
  const int K0 = n;
  // NaN wants: such a row's threshold has W + s in its wantExtra (its w > deservedShare
  // is false), not one of T(s) below -- k_general collects the rows' own thresholds
  bool bad = K0 > kHetMaxS || st.a.nan;
  if (!bad) {
    for (int i = t; i < 2 * kHetMaxS; i += 256)
      if (set[i] != kHetEmpty) {
        const double s = (double)set[i];
        const double eq = st.rs.C / (double)st.cl.count;  // as fs_stage01's arguments
        const double ds = eq * s;                          // :126
        const double dE = (b.x / (double)b.i) * s;         // :175 (wantExtra = W for a round-2 row)
        T[atomicAdd(&fill, 1)] = dE + ds;                  // :197
      }
    __syncthreads();
    if (t >= K0) T[t] = __builtin_inf();
    int nonfinite = 0;
    if (t < K0 && !__builtin_isfinite(T[t])) nonfinite = 1;
    bad = __syncthreads_or(nonfinite) != 0;
  }
  if (bad) {  // k_general decides the resource (per-threshold passes)
    if (t == 0) {
      H->mode = 2;
      general_list[atomicAdd(general_count, 1)] = L.seg;
    }
    return;
  }
  for (int k = 2; k <= kHetMaxS; k <<= 1)  // ascending bitonic sort of the thresholds
    for (int j = k >> 1; j > 0; j >>= 1) {
      __syncthreads();
      const int q = t ^ j;
      if (q > t) {
        const double x = T[t], y = T[q];
        if ((x > y) == ((t & k) == 0)) {
          T[t] = y;
          T[q] = x;
        }
      }
    }
  __syncthreads();
  if (t == 0) {  // distinct values only (counts may share a threshold)
    int K = 0;
    for (int i = 0; i < K0; ++i)
      if (K == 0 || T[i] != H->T[K - 1]) H->T[K++] = T[i];
    H->K = K;
    H->mode = 1;
  }
}

// One 64-row tile of a wave into its bucket accumulators (k_general's method:
// sort the lanes by bucket, segmented scan, one writer per bucket; fixed order).
__device__ __forceinline__ void het_tile(const double* T, int K, double w, long long s, bool in, double* accw,
                                         long long* accs, int* accc) {
  const int lane = threadIdx.x & 63;
  const uint32_t bk = in ? (uint32_t)gen_bucket(T, K, w) : 0xFFFFu;
  const uint32_t key = wave_sort64(bk << 6 | (uint32_t)lane);
  const int src = (int)(key & 63);
  const int mb = (int)(key >> 6);
  double vw = shfl_d(in ? w : 0.0, src);
  long long vs = __shfl(in ? s : 0ll, src, 64);
  int vc = mb != 0xFFFF ? 1 : 0;
  const int prevb = __shfl_up(mb, 1, 64);
  int run = (lane == 0 || prevb != mb) ? 1 : 0;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double ow = shfl_d(vw, lane >= off ? lane - off : lane);
    const long long os = __shfl(vs, lane >= off ? lane - off : lane, 64);
    const int oc = __shfl(vc, lane >= off ? lane - off : lane, 64);
    const int orun = __shfl(run, lane >= off ? lane - off : lane, 64);
    if (lane >= off && !run) {
      vw = ow + vw;
      vs = os + vs;
      vc = oc + vc;
      run = orun;
    }
  }
  const int nextb = __shfl_down(mb, 1, 64);
  if (mb != 0xFFFF && (lane == 63 || nextb != mb)) {
    accw[mb] += vw;
    accs[mb] += vs;
    accc[mb] += vc;
  }
}

__global__ __launch_bounds__(256) void k_large_c_het(DevParams p, const Chunk* __restrict__ chunks,
                                                     const LargeSeg* __restrict__ ls, Partials P) {
  __shared__ double T[kHetMaxS];
  __shared__ double accw[4][kHetBuckets];
  __shared__ long long accs[4][kHetBuckets];
  __shared__ int accc[4][kHetBuckets];
  const int t = threadIdx.x, wv = t >> 6;
  const Chunk ch = chunks[blockIdx.x];
  const HetRes* H = het_of(P, ch.lseg);
  if (H->mode != 1) return;
  ChunkRows rw;
  load_chunk_w(p, P, ch, rw, true);
  const SegState st = seg_state_of(p, ch.seg, seg_tot(P, ch.lseg)->a);
  const double eq = st.rs.C / (double)st.cl.count;
  const int K = H->K;
  for (int i = t; i < K; i += 256) T[i] = H->T[i];
  for (int i = t; i < 4 * kHetBuckets; i += 256) {
    (&accw[0][0])[i] = 0.0;
    (&accs[0][0])[i] = 0;
    (&accc[0][0])[i] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kLR; ++k) {  // row k*256 + t: tile 4k + wv, in order per wave
    const double w = rw.w[k];
    const long long s = rw.s[k];
    const bool in = (rw.live >> k & 1) && w > (double)s * eq;  // wantExtraClients (:165-169)
    het_tile(T, K, w, s, in, accw[wv], accs[wv], accc[wv]);
  }
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * kHetBuckets;
  for (int bb = t; bb < 2 * K + 1; bb += 256) {  // the waves combined in a fixed order
    P.bk_w[base + bb] = ((accw[0][bb] + accw[1][bb]) + accw[2][bb]) + accw[3][bb];
    P.bk_s[base + bb] = accs[0][bb] + accs[1][bb] + accs[2][bb] + accs[3][bb];
    P.bk_c[base + bb] = accc[0][bb] + accc[1][bb] + accc[2][bb] + accc[3][bb];
  }
}

// one wave per (resource, bucket): the bucket's chunk partials, lanes striding the
// chunks, combined by the fixed DPP tree of wave_reduce
__global__ __launch_bounds__(256) void k_large_e(DevParams p, const LargeSeg* __restrict__ ls, Partials P) {
  const int lane = threadIdx.x & 63;
  const LargeSeg L = ls[blockIdx.x];
  HetRes* H = het_of(P, blockIdx.x);
  if (H->mode != 1) return;
  const int bb = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (bb >= 2 * H->K + 1) return;  // whole waves
  AggR v{0, 0.0, 0.0};  // cnt: clients, h: subclients (exact below 2^53), w: wants
  for (int q = L.chunk_begin + lane; q < L.chunk_end; q += 64) {
    const size_t i = (size_t)q * kHetBuckets + bb;
    v.w += P.bk_w[i];
    v.h += (double)P.bk_s[i];
    v.cnt += P.bk_c[i];
  }
  v = wave_reduce(v, OpR());
  if (lane == 0) {
    H->bw[bb] = v.w;
    H->bs[bb] = (int64_t)v.h;
    H->bc[bb] = v.cnt;
  }
}

__global__ __launch_bounds__(256) void k_large_map_het(DevParams p, const Chunk* __restrict__ chunks,
                                                       const LargeSeg* __restrict__ ls, Partials P) {
  __shared__ Lds<256> lds;
  __shared__ double T[kHetMaxS], ee[kHetMaxS];
  __shared__ long long sgt[kHetMaxS];
  const int t = threadIdx.x;
  const Chunk ch = chunks[blockIdx.x];
  const HetRes* H = het_of(P, ch.lseg);
  if (H->mode != 1) return;
  ChunkRows rw;
  load_chunk_w(p, P, ch, rw, true, true);
  const SegTot* tot = seg_tot(P, ch.lseg);
  const SegState st = seg_state_of(p, ch.seg, tot->a);
  const AggB b = tot->b;
  const double C = st.rs.C;
  const double eq = C / (double)st.cl.count;
  const int K = H->K;
  __shared__ double bw[kHetBuckets];
  __shared__ long long bs[kHetBuckets], bc[kHetBuckets];
  for (int i = t; i < K; i += 256) T[i] = H->T[i];
  for (int i = t; i < 2 * K + 1; i += 256) {
    bw[i] = H->bw[i];
    bs[i] = H->bs[i];
    bc[i] = H->bc[i];
  }
  __syncthreads();
  if (t == 0) {  // prefix over the buckets (as k_general): every chunk the same, in LDS
    long long stot = 0;
    for (int bb = 0; bb < 2 * K + 1; ++bb) stot += bs[bb];
    long long cnt = 0, sle = 0;
    double sw = 0.0;
    for (int k = 0; k < K; ++k) {
      const int bl = 2 * k;  // below T_k; bl + 1: w == T_k
      cnt += bc[bl];
      sw = sw + bw[bl];
      sle += bs[bl];
      const long long seq = bs[bl + 1];
      ee[k] = cnt == 0 ? 0.0 : (double)cnt * T[k] - sw;  // :197-198
      sgt[k] = stot - sle - seq;                          // :199-200
      sle += seq;
      cnt += bc[bl + 1];
      sw = sw + bw[bl + 1];
    }
  }
  __syncthreads();
  SumD delta{0.0};
#pragma unroll
  for (int k = 0; k < kLR; ++k) {
    if (!(rw.valid >> k & 1)) continue;
    const unsigned u = (unsigned)(k * 256 + t);
    const double w = rw.w[k], h = rw.h[k];
    if (!(rw.live >> k & 1)) {
      put_released<kSpecNT>(p, ch.row0, u, (rw.rel >> k & 1) ? (int32_t)kSubReleased : 0);
      continue;
    }
    const long long s = rw.s[k];
    double g, Tr = 0.0;
    if (!fs_stage01(w, h, s, C, st.cl.sum_has, eq, b.x, b.i, &g, &Tr)) {
      AggC c{0.0, 0};
      if (!__builtin_isnan(Tr)) {
        const int q = gen_index(T, K, Tr);
        c = AggC{ee[q], sgt[q]};
      }
      g = fs_stage2(w, h, s, C, st.cl.sum_has, eq, b.x, b.i, Tr, c);
    }
    put_live<kSpecNT>(p, ch.row0, u, g, st.rs, (rw.expl >> k & 1) ? (p.sub[ch.row0 + u] | (int32_t)kSubExplicit) : 0);
    delta.v += g - h;
  }
  delta = group_reduce<256>(delta, OpSumD(), lds.d);
  if (t == 0) P.d_delta[blockIdx.x] = delta.v;
}

// --------------------------------------------------------------------------
// store maintenance
// --------------------------------------------------------------------------
// Assign on existing rows (store.go:153-167): running sums += new - old.
// Rows of one call may hit the same resource, so the deltas reach the sums
// through atomics — one per run of a resource within a wave (wave_seg_add).
// resource owning row r: last s with seg_off[s] <= r.  A coarse index (the
// resource holding the first row of every 2^kRowBlkShift-row block) narrows the
// binary search to the few resources of r's block.
__device__ __forceinline__ int seg_of_row(const RowIndex& ix, int64_t r) {
  const int64_t* __restrict__ seg_off = ix.seg_off;
  const int64_t b = r >> kRowBlkShift;
  int64_t lo = ix.blk_seg[b];
  int64_t hi = (int64_t)ix.blk_seg[b + 1] + 1;  // invariant: seg_off[lo] <= r < seg_off[hi]
  if (hi > ix.R) hi = ix.R;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= r)
      lo = mid;
    else
      hi = mid;
  }
  return (int)lo;
}

// Add per-row deltas to their resources' running sums: lanes of a wave that hit
// the same resource are summed first (DPP) and add once; a wave whose rows spread
// over many resources adds per lane.  Every lane of the wave must call this.
__device__ __forceinline__ void wave_seg_add(ResAgg* agg, bool active, int seg, double dh, double dw, long long ds,
                                             bool with_has, bool with_count) {
  const int lane = threadIdx.x & 63;
  const unsigned long long act = __ballot(active);
  const int prev = __shfl(seg, lane > 0 ? lane - 1 : 0, 64);
  const bool head = active && (lane == 0 || !((act >> (lane - 1)) & 1) || prev != seg);
  if (__popcll(__ballot(head)) > 8) {
    if (active) {
      if (with_has) atomicAdd(&agg[seg].sum_has, dh);
      atomicAdd(&agg[seg].sum_wants, dw);
      if (with_count) atomicAdd((unsigned long long*)&agg[seg].count, (unsigned long long)ds);
    }
    return;
  }
  unsigned long long rem = act;
  while (rem) {
    const int h = __builtin_ctzll(rem);
    const int s0 = __builtin_amdgcn_readlane(seg, h);
    const unsigned long long m = __ballot(active && seg == s0) & rem;
    const bool in = (m >> lane) & 1;
    AggR v{in ? ds : 0, in ? dh : 0.0, in ? dw : 0.0};
    v = wave_reduce(v, OpR());
    if (lane == h) {
      if (with_has) atomicAdd(&agg[s0].sum_has, v.h);
      atomicAdd(&agg[s0].sum_wants, v.w);
      if (with_count) atomicAdd((unsigned long long*)&agg[s0].count, (unsigned long long)v.cnt);
    }
    rem &= ~m;
  }
}

// Validation of one store-update call on the device (no O(n) host pass): rows in
// range and unique within the call (a row bitmap, all-zero between calls), and
// the value flags the planner needs.  The apply kernels run only if no error bit
// is set, so a rejected call leaves the store untouched.
__global__ void k_check_rows(int64_t n, const int64_t* __restrict__ rows, int64_t N, uint32_t* bitmap,
                             const double* __restrict__ wants, const int64_t* __restrict__ sub,
                             const int32_t* __restrict__ sub32, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t f = 0;
  if (i < n) {
    const int64_t r = rows[i];
    if (r < 0 || r >= N) {
      f |= kUpdRange;
    } else {
      const uint32_t bit = 1u << (r & 31);
      if (atomicOr(&bitmap[r >> 5], bit) & bit) f |= kUpdDup;
    }
    if (wants && __builtin_isnan(wants[i])) f |= kUpdNaN;
    if (sub || sub32) {
      const int64_t v = sub32 ? (int64_t)sub32[i] : sub[i];
      if (v < 0 || v > kSubMax) f |= kUpdSub;
      if (v != 1) f |= kUpdNotOne;
    }
  }
  // one atomic per wave and flag value
  const uint32_t lo = __builtin_amdgcn_readfirstlane(f);
  if (__all(f == lo)) {
    if ((threadIdx.x & 63) == 0 && lo) atomicOr(flags, lo);
  } else if (f) {
    atomicOr(flags, f);
  }
}

// Return the bitmap words of this call's rows to zero.
__global__ void k_clear_rows(int64_t n, const int64_t* __restrict__ rows, int64_t N, uint32_t* bitmap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  if (r >= 0 && r < N) bitmap[r >> 5] = 0u;
}

// Narrow arrivals (dm_store_batch): has == nullptr -> 0; sub32 instead of sub;
// expiry == nullptr -> the resource's now + lease length (the Assign's expiry,
// store.go:161).
// one byte of a dense resource's masks (dm_device.h mask_pos), atomically: rows of one
// resource share the mask words
__device__ __forceinline__ void mask_bit(uint8_t* base, int32_t off, int32_t bit, bool set) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(base + off);
  unsigned* w = reinterpret_cast<unsigned*>(a & ~uintptr_t(3));
  const unsigned m = 1u << (bit + 8 * (int)(a & 3));
  if (set)
    atomicOr(w, m);
  else
    atomicAnd(w, ~m);
}

// The row's place in its dense resource's masks, or false when the resource is not in
// a dense state its item describes (dm_device.h DenseUpd).
__device__ __forceinline__ bool dense_row(const DenseUpd& du, const RowIndex& ix, int seg, int64_t r, uint8_t state,
                                          MaskPos* mp, WorkItem** item) {
  if (state < 2 || !du.item_of) return false;
  const int32_t io = du.item_of[seg];
  if (io < 0) return false;
  const int bin = io >> 24;
  WorkItem* it = du.bins[bin - 3] + (io & 0xFFFFFF);
  if (((it->n >> 16) & 0xFF) != state - 1) return false;  // the hint is the state's (a new shape clears hints)
  int G, R;
  bin_shape(bin, du.bin4_wave, du.bin6_wide, &G, &R);
  const int64_t lo = ix.seg_off[seg];
  *mp = mask_pos(G, R, (int)(r - lo));
  *item = it;
  return true;
}

__global__ void k_upsert(int64_t n, const int64_t* __restrict__ rows, const double* __restrict__ has,
                         const double* __restrict__ wants, const int64_t* __restrict__ sub,
                         const int32_t* __restrict__ sub32, const int64_t* __restrict__ expiry,
                         const ResCfg* __restrict__ cfg, int64_t now, RowIndex ix, double* s_has, double* s_wants,
                         int32_t* s_sub, int64_t* s_exp, ResAgg* agg, uint8_t* expl, const uint32_t* flags,
                         DenseUpd du) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (*flags & kUpdReject) return;  // uniform over the grid
  const bool active = i < n;
  int seg = 0;
  double dh = 0.0, dw = 0.0;
  long long ds = 0;
  if (active) {
    const int64_t r = rows[i];
    seg = seg_of_row(ix, r);
    const double hv = has ? has[i] : 0.0;
    const int64_t sv = sub32 ? (int64_t)sub32[i] : sub[i];
    dh = hv - s_has[r];
    dw = wants[i] - s_wants[r];
    ds = sv - sub_value(s_sub[r]);
    s_has[r] = hv;
    s_wants[r] = wants[i];
    s_sub[r] = (int32_t)((uint32_t)sv | kSubExplicit);  // in [0, kSubMax] (k_check_rows); expiry explicit
    const int64_t ex = expiry ? expiry[i] : now + (int64_t)cfg[seg].lease_len_s * kNs;
    s_exp[r] = ex;
    // an arrival with the dense resource's count and the Assign's expiry, not before the
    // followers': the resource stays dense, the row goes into its arrival mask
    MaskPos mp;
    WorkItem* it;
    const uint8_t st = expl[seg];
    if (!expiry && dense_row(du, ix, seg, r, st, &mp, &it) && sv == (int64_t)st - 1 && ex >= agg[seg].follow_exp) {
      mask_bit(du.rmask + rel_mask_offset(ix.seg_off[seg]), mp.roff, mp.rbit, false);
      mask_bit(du.rmask + rel_mask_offset(ix.seg_off[seg]), mp.aoff, mp.abit, true);
      atomicOr(&it->n, 1 << 25);
    } else {
      expl[seg] = 1;  // the tick reads this resource's expiry column again
    }
  }
  wave_seg_add(agg, active, seg, dh, dw, ds, true, true);
}

__global__ void k_release(int64_t n, const int64_t* __restrict__ rows, RowIndex ix, double* s_has, double* s_wants,
                          int32_t* s_sub, int64_t* s_exp, ResAgg* agg, uint8_t* expl, const uint32_t* flags,
                          DenseUpd du) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (*flags & kUpdReject) return;  // uniform over the grid
  const bool active = i < n;
  int seg = 0;
  double dh = 0.0, dw = 0.0;
  long long ds = 0;
  if (active) {
    const int64_t r = rows[i];
    seg = seg_of_row(ix, r);
    dh = -s_has[r];
    dw = -s_wants[r];
    ds = -(long long)sub_value(s_sub[r]);
    s_has[r] = 0.0;
    s_wants[r] = 0.0;
    s_sub[r] = (int32_t)kSubReleased;  // the mark every reader decodes first: the expiry column is left alone
    (void)s_exp;
    MaskPos mp;
    WorkItem* it;
    const uint8_t st = expl[seg];
    if (dense_row(du, ix, seg, r, st, &mp, &it)) {  // stays dense: the row into the released-row mask
      uint8_t* mb = du.rmask + rel_mask_offset(ix.seg_off[seg]);
      mask_bit(mb, mp.roff, mp.rbit, true);
      mask_bit(mb, mp.aoff, mp.abit, false);  // (a row that arrived since the last tick)
      atomicOr(&it->n, 1 << 24);
    } else if (st >= 2) {
      expl[seg] = 0;  // no longer dense: the next tick reads the subclients column
    }
  }
  wave_seg_add(agg, active, seg, dh, dw, ds, true, true);
}

// Narrow Assign for a refresh that only changes wants (store.go:157):
// sumWants += new - old.  Rows are unique within one call.
// A released row is a free slot, not a client: a refresh of it changes nothing (a
// returning client is an arrival, dm_store_upsert).  Written into it, the wants would
// be subtracted from the resource's running sum by every later tick's Clean.
__global__ void k_update_wants(int64_t n, const int64_t* __restrict__ rows, const double* __restrict__ wants,
                               RowIndex ix, const int32_t* __restrict__ s_sub, double* s_wants, ResAgg* agg,
                               const uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (*flags & kUpdReject) return;  // uniform over the grid
  const bool active = i < n;
  int seg = 0;
  double d = 0.0;
  if (active) {
    const int64_t r = rows[i];
    seg = seg_of_row(ix, r);
    if (!sub_released(s_sub[r])) {
      d = wants[i] - s_wants[r];
      s_wants[r] = wants[i];
    }
  }
  wave_seg_add(agg, active, seg, 0.0, d, 0, false, false);
}

// ---- wants updates as a row mask + packed values (dm_store_update_wants_mask) ----
// Bit j of word w is row first_row + 64 w + j; the set rows take the packed values
// in ascending row order.  At 10% of the rows updated this moves 1.25 B of mask
// per update over PCIe instead of an 8-B row index (C4: 116 instead of 200 MB).
struct OpAddI64 {
  __device__ long long operator()(long long a, long long b) const { return a + b; }
};
// Pass 1: popcount per 256-word block (+ rows past the store's end), and every
// word's exclusive offset within its block.
__global__ __launch_bounds__(256) void k_mask_count(int64_t nwords, const uint64_t* __restrict__ mask,
                                                    int64_t first_row, int64_t N, int64_t* block_sums,
                                                    int32_t* word_pre, uint32_t* flags) {
  __shared__ int part[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t m = w < nwords ? mask[w] : 0ull;
  const int64_t row0 = first_row + 64 * w;
  if (m && row0 + 63 >= N) {  // bits of rows >= N
    const int64_t keep = N - row0;  // < 64
    const uint64_t ok = keep <= 0 ? 0ull : ((1ull << keep) - 1ull);
    if (m & ~ok) atomicOr(flags, kUpdRange);
  }
  const int c = __popcll(m);
  int incl = c;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) part[wave] = incl;
  __syncthreads();
  int pre = incl - c;
  for (int i = 0; i < wave; ++i) pre += part[i];
  if (w < nwords) word_pre[w] = pre;
  if (threadIdx.x == 0) block_sums[blockIdx.x] = (int64_t)part[0] + part[1] + part[2] + part[3];
}

// Pass 2 (one workgroup): exclusive scan of the block sums in place; the total
// must equal the number of packed values.
__global__ __launch_bounds__(1024) void k_mask_scan(int64_t nblocks, int64_t* block_sums, int64_t n_values,
                                                    uint32_t* flags) {
  __shared__ int64_t tot[1024];
  const int t = threadIdx.x;
  const int64_t per = (nblocks + 1023) / 1024;
  const int64_t b0 = t * per < nblocks ? t * per : nblocks;
  const int64_t b1 = b0 + per < nblocks ? b0 + per : nblocks;
  int64_t s = 0;
  for (int64_t b = b0; b < b1; ++b) s += block_sums[b];
  tot[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan of the 1024 partials
    const int64_t v = t >= o ? tot[t - o] : 0;
    __syncthreads();
    tot[t] += v;
    __syncthreads();
  }
  int64_t run = tot[t] - s;
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t v = block_sums[b];
    block_sums[b] = run;
    run += v;
  }
  if (t == 1023 && tot[1023] != n_values) atomicOr(flags, kUpdCount);
}

// Pass 3: one lane per row; a wave takes kMaskWords consecutive mask words (64
// rows each).  Lane q first fetches word q, its first value's offset and the
// resource of its first row (all words in parallel); then every row's loads of
// every word are issued before any is consumed (coalesced: per word the wave reads
// its packed values and 512 B of the wants column).  A resource's deltas stay in
// per-lane registers while consecutive words lie inside it and leave with one
// reduction + atomic when the resource changes; a word that spans resources adds
// its runs directly (wave_seg_add).
constexpr int kMaskWords = 16;
__global__ __launch_bounds__(256) void k_mask_apply(int64_t nwords, const uint64_t* __restrict__ mask,
                                                    int64_t first_row, const int64_t* __restrict__ block_offs,
                                                    const int32_t* __restrict__ word_pre,
                                                    const double* __restrict__ wants, RowIndex ix,
                                                    const int32_t* __restrict__ s_sub, double* s_wants, ResAgg* agg,
                                                    uint32_t* flags, int64_t vlo, int64_t vhi) {
  if (*flags & kUpdReject) return;  // uniform over the grid
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kMaskWords;
  if (w0 >= nwords) return;  // whole waves
  const int nw = nwords - w0 < kMaskWords ? (int)(nwords - w0) : kMaskWords;
  uint64_t my_m = 0ull;
  int64_t my_off = 0, my_end = 0;
  if (lane < nw) {
    const int64_t w = w0 + lane;
    my_m = mask[w];
    my_off = block_offs[w >> 8] + word_pre[w];
  }
  // only the values [vlo, vhi) have landed (dm_store_apply copies them in chunks): a
  // wave whose words' values all lie outside is done
  {
    const int64_t first = readlane_any(my_off, 0);
    const int64_t last = readlane_any(my_off, nw - 1) + __popcll(readlane_any(my_m, nw - 1));  // one past
    if (last <= vlo || first >= vhi) return;
  }
  int my_seg = 0;
  if (lane < nw) {
    my_seg = seg_of_row(ix, first_row + 64 * (w0 + lane));
    my_end = ix.seg_off[my_seg + 1];  // the word lies in one resource iff its last row < my_end
  }
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t inr = 0;  // bit q: this lane's row of word q is set and its value in [vlo, vhi)
  double v[kMaskWords], old[kMaskWords];
  uint32_t freed = 0;  // bit q: this lane's row of word q is released (k_update_wants: left alone)
#pragma unroll
  for (int q = 0; q < kMaskWords; ++q) {  // every load in flight before the first use
    v[q] = 0.0;
    old[q] = 0.0;
    if (q < nw) {
      const uint64_t m = readlane_any(my_m, q);
      const int64_t vi = readlane_any(my_off, q) + __popcll(m & below);
      if (((m >> lane) & 1ull) && vi >= vlo && vi < vhi) {
        inr |= 1u << q;
        v[q] = wants[vi];
        old[q] = s_wants[first_row + 64 * (w0 + q) + lane];
        freed |= (sub_released(s_sub[first_row + 64 * (w0 + q) + lane]) ? 1u : 0u) << q;
      }
    }
  }
  int cur = -1;      // resource whose deltas `acc` holds (uniform)
  double acc = 0.0;  // this lane's share of them
  bool nan = false;
#pragma unroll
  for (int q = 0; q < kMaskWords; ++q) {
    const uint64_t m = q < nw ? readlane_any(my_m, q) : 0ull;
    if (m != 0ull) {  // uniform
      const int64_t row0 = first_row + 64 * (w0 + q);
      const bool act = (inr >> q & 1u) && !(freed >> q & 1u);
      const int s0 = __builtin_amdgcn_readlane(my_seg, q);
      const bool single = readlane_any(my_end, q) > row0 + 63 - __builtin_clzll(m);
      double d = 0.0;
      int seg = s0;
      if (act) {
        const int64_t r = row0 + lane;
        nan |= __builtin_isnan(v[q]);
        if (!single)
          while (ix.seg_off[seg + 1] <= r) ++seg;
        d = v[q] - old[q];
        s_wants[r] = v[q];
      }
      if (single && s0 == cur) {
        acc += d;
      } else {
        if (cur >= 0) {  // flush the previous resource
          const double t = wave_reduce(acc, [](double a, double b) { return a + b; });
          if (lane == 0) atomicAdd(&agg[cur].sum_wants, t);
        }
        if (single) {
          cur = s0;
          acc = d;
        } else {
          cur = -1;
          acc = 0.0;
          wave_seg_add(agg, act, seg, 0.0, d, 0, false, false);
        }
      }
    }
  }
  if (cur >= 0) {
    const double t = wave_reduce(acc, [](double a, double b) { return a + b; });
    if (lane == 0) atomicAdd(&agg[cur].sum_wants, t);
  }
  if (__ballot(nan) && lane == 0) atomicOr(flags, kUpdNaN);
}

// dm_store_apply: a part is applied only if no earlier part was rejected.
__global__ void k_carry_reject(const uint32_t* __restrict__ from, uint32_t* to) { *to |= *from & kUpdReject; }

// gets / expiry of scattered rows (dm_read_leases_rows)
// Rows as the store holds them (dm_device.h encoding), for the host: the expiry of
// row r (a follower's is its resource's follow_exp) and its subclients value.
// rows == nullptr: rows off .. off+n-1.
__global__ void k_resolve_rows(int64_t n, const int64_t* __restrict__ rows, int64_t off, const int32_t* __restrict__ sub,
                               const int64_t* __restrict__ expiry, RowIndex ix, const ResAgg* __restrict__ agg,
                               int64_t* out_exp, int64_t* out_sub) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows ? rows[i] : off + i;
  const int32_t raw = sub[r];
  int64_t e;
  if (sub_released(raw))
    e = kReleased;
  else if (raw < 0)
    e = expiry[r];
  else
    e = agg[seg_of_row(ix, r)].follow_exp;
  if (out_exp) out_exp[i] = e;
  if (out_sub) out_sub[i] = sub_value(raw);
}

__global__ void k_gather_leases(int64_t n, const int64_t* __restrict__ rows, const double* __restrict__ gets,
                                const int64_t* __restrict__ expiry, double* out_gets, int64_t* out_exp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  out_gets[i] = gets[r];
  if (expiry) out_exp[i] = expiry[r];  // else resolved by k_resolve_rows
}

// server.go:234-255: what an intermediate server sends upstream -- {SumWants, Count}
// of every resource it holds (a band only when SumWants > 0, :241) -- plus the root's
// validation of that request (:858-868), computed here once instead of by every
// root copy: a band with Count < 1 fails the whole GetServerCapacity with
// InvalidArgument (:863-866), and a Count beyond the root's 32-bit subclients
// column is rejected the same way (kHierCountRange).  dst[1 + r] = the record of
// resource r; dst[0] = {the flags of the whole request, 0}, written by the last
// workgroup to arrive (sync[0] accumulates the workgroups' flags, sync[1] counts
// them; both return to zero for the next launch).
__global__ __launch_bounds__(256) void k_publish(int64_t R, const ResAgg* __restrict__ agg, double2* __restrict__ dst,
                                                 uint32_t* sync, int nblocks) {
  __shared__ uint32_t wf[4];
  uint32_t f = 0;
  // a few workgroups striding over the records: each one arrives at the counter once
  // (hundreds of contended arrivals cost ~10 us per launch at R = 100k)
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < R; r += (int64_t)nblocks * 256) {
    const ResAgg a = agg[r];
    double2 v;
    v.x = a.sum_wants;
    v.y = __longlong_as_double(a.count);
    dst[1 + r] = v;
    if (a.sum_wants > 0.0) {  // a band (server.go:241)
      if (a.count < 1) f |= kHierInvalid;
      if (a.count > kSubMax) f |= kHierCountRange;
    }
  }
  const uint32_t w = (__ballot(f & kHierInvalid) ? kHierInvalid : 0u) | (__ballot(f & kHierCountRange) ? kHierCountRange : 0u);
  if ((threadIdx.x & 63) == 0) wf[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0) {
      const uint32_t all = wf[0] | wf[1] | wf[2] | wf[3];
      if (all) (void)__hip_atomic_fetch_or((gu32*)sync, all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (arrive_last(sync + 1, nblocks) && threadIdx.x == 0) {
      const uint32_t flags = __hip_atomic_load((gu32*)sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32*)sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      double2 v;
      v.x = __longlong_as_double((long long)flags);
      v.y = 0.0;
      dst[0] = v;
    }
  }
}

// One exchange round of the root.  The requests of the servers that ask for a
// resource -- {has 0 (the intermediate never fills Has, server.go:244,873), wants
// SumWants_g, subclients Count_g} -- are decided by Resource.Decide one after
// another in server order, as the root's res.mu serialises the GetServerCapacity
// calls (resource.go:103-104): Clean once (resource.go:106, store.go:169-181;
// nothing else expires within the round), then per request Learn or the algorithm
// (algorithm.go:95-302, with the request's own values for its server) against
// the store as the Assigns of the earlier requests left it, then its Assign
// (store.go:153-167: the row and the running sums).  So the root never grants
// more than the reference would: a FairShare resource with capacity C and G
// servers that each want C grants C, 0, ... in the first round, not G x C.
// Servers that do not request keep their root lease until Clean expires it.  The
// running sums follow the reference's update sequence -- Clean's releases in row
// order, then one Assign per request in server order -- bit for bit.
//
// Layouts (HierArgs): replicated -- every server holds every resource, the root
// store has K = G rows per resource (row r*G + g = server g); sharded -- server g
// holds resources [lo[g], lo[g+1]) (contiguous resource-id ranges),
// so only the owner ever requests resource r and the root store has one row per
// resource (K = 1); there each rank decides only its own range [r_lo, r_hi): no
// other server requests those resources and no other resource's root rows reach this
// server's leaf, so the launch shrinks with the shard (the other ranks decide theirs).
// A server whose published flags are set (a band with
// num_clients < 1, server.go:863-866, or a Count beyond 2^31 - 2) requests nothing
// this round.
//
// K <= 64 rows: a wave holds 64 / P whole resources (P = K rounded up to a power
// of two), one lane per row.  For each row q in order, the lanes of a resource
// walk its rows in row order by shuffles for the decision's loops over store.Map
// (round 1, round 2, ProportionalShare's extra capacity / need: the sums of a
// sequential Map, bit for bit the oracle's); lane q then takes the Assign.  O(K)
// per decision, K decisions per resource.
// The lane of `ha.server` then writes that server's template for each of its
// resources exactly as performRequests + LoadConfig do (server.go:279-313,
// resource.go:117-125): a requested resource takes the root's grant as capacity,
// its expiry (Unix seconds) as the parent expiry, and the root's algorithm
// (kind, lease length, refresh) and configured safe capacity (0 when unset,
// server.go:894); a resource it did not request drops to the "*" default
// template (server.go:53-63: capacity 0, safe 0, FAIR_SHARE, lease 20 s, refresh
// 1 s, no parent expiry); a rejected round keeps the templates it had
// (performRequests returns before LoadConfig, :268-272).  learningModeEndTime is
// kept (set once, resource.go:163).
__device__ __forceinline__ int hier_owner(const int64_t* lo, int G, int64_t r) {
  int a = 0, b = G;  // lo[a] <= r < lo[b]
  while (b - a > 1) {
    const int m = (a + b) >> 1;
    if (lo[m] <= r) a = m;
    else b = m;
  }
  return a;
}

__global__ __launch_bounds__(256) void k_hier_tick(DevParams p, HierArgs ha) {
  const int K = ha.K;
  const int P = K <= 1 ? 1 : 1 << (32 - __builtin_clz((unsigned)(K - 1)));
  const int per = 64 / P;  // resources per wave
  const int lane = threadIdx.x & 63;
  const int rl = lane / P, g0 = lane - rl * P;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x < ha.G)  // the round's per-server flags (dm_hier_status)
    ha.status_out[threadIdx.x] = pub_flags(ha.gathered[(int64_t)threadIdx.x * ha.stride].x);
  const int64_t r = ha.r_lo + wave * per + rl;
  if (ha.r_lo + wave * per >= ha.r_hi) return;  // whole waves only
  const bool valid = g0 < K && r < ha.r_hi;
  const int64_t rr = r < ha.r_hi ? r : ha.r_lo;
  const int64_t row = rr * K + (valid ? g0 : 0);
  // the server this row belongs to, and its record of the resource
  const int g = ha.shard_lo ? hier_owner(ha.shard_lo, ha.G, rr) : g0;
  const int64_t rec = ha.shard_lo ? rr - ha.shard_lo[g] : rr;
  double w = 0.0, h = 0.0, rw = 0.0;
  int s = 0, rs = 0;
  int64_t e = kReleased;
  bool req = false;
  uint32_t flags = 0;
  const Res rs_cfg = load_res(p, (int)rr);
  // every load the round needs is issued here, before the first is consumed: the
  // expiry column (root rows are explicit; read unconditionally instead of after the
  // subclients word) and this server's template inputs (one round trip instead of three)
  const bool mine = valid && g == ha.server;
  const int64_t li = mine ? rr - ha.leaf_lo : 0;  // the resource's index in this server's leaf
  int64_t learn = 0;
  ResCold rcc{0.0, 0, 0};
  if (mine) {
    learn = ha.leaf_prev_cfg[li].learning_end_ns;  // kept (resource.go:163)
    rcc = ha.root_cold[rr];
  }
  if (valid) {
    w = p.wants[row];
    h = p.has[row];
    const int32_t raw = p.sub[row];  // expiry encoding (dm_device.h): root rows are explicit or released
    const int64_t xe = p.expiry[row];
    s = sub_value(raw);
    e = sub_released(raw) ? kReleased : (raw < 0 ? xe : rs_cfg.follow_exp);
    const double2* blk = ha.gathered + (int64_t)g * ha.stride;
    flags = pub_flags(blk[0].x);
    const double2 v = blk[1 + rec];
    req = flags == 0u && v.x > 0.0;  // count in [1, kSubMax] when the flags are clear
    rw = v.x;
    rs = req ? (int)__double_as_longlong(v.y) : 0;
  }
  const bool released = e == kReleased;
  bool live = valid && !released && !(p.now > e);          // present after Clean (store.go:174)
  const bool expired = valid && !released && (p.now > e);  // released by this round's Clean
  const int base = rl * P;                                 // first lane of this resource
  auto src = [&](int q) { return base + q; };

  // Clean on the running sums, in row order (store.go:169-181 -> :142-151)
  long long count = rs_cfg.agg_count;
  double sh = rs_cfg.agg_has, sw = rs_cfg.agg_wants;
  const int xp = expired ? 1 : 0;
  if (__any(xp)) {
    for (int q = 0; q < K; ++q) {
      const double hj = shfl_d(h, src(q)), wj = shfl_d(w, src(q));
      const int sj = shfl_i(s, src(q)), xj = shfl_i(xp, src(q));
      if (xj) {
        sw -= wj;
        sh -= hj;
        count -= sj;
      }
    }
  }
  if (!live) {  // this row is absent from the store the round starts with
    h = 0.0;
    w = 0.0;
    s = 0;
  }

  const double C = rs_cfg.C;
  const bool ps = !rs_cfg.learning && rs_cfg.kind == 2;
  const int rq = req ? 1 : 0;
  double my_gets = 0.0;
  for (int q = 0; q < K; ++q) {
    const int rq_q = shfl_i(rq, src(q));
    if (!__any(rq_q)) continue;  // no resource of this wave has server q's request
    const double rw_q = shfl_d(rw, src(q));
    const int rs_q = shfl_i(rs, src(q));
    const int live_q = shfl_i(live ? 1 : 0, src(q));
    const double old_h = shfl_d(h, src(q)), old_w = shfl_d(w, src(q));  // store.Get: zero when absent
    const int old_s = shfl_i(s, src(q));
    // Decide (algorithm.go) for server q's request against the store as it is now
    double gets = 0.0, eq = 0.0, ds = 0.0, avail = 0.0;
    bool loop1 = false;
    if (rq_q) {
      if (rs_cfg.learning) {
        gets = 0.0;  // Learn: the request's Has (never filled by an intermediate)
      } else if (rs_cfg.kind == 0) {
        gets = rw_q;
      } else if (rs_cfg.kind == 1) {
        gets = minF(C, rw_q);
      } else if (ps) {
        const long long cnt = count + (live_q ? 0 : rs_q);  // :217-225
        eq = C / (double)cnt;                               // :229
        ds = eq * (double)rs_q;                             // :233 equalSharePerClient
        avail = C - sh + old_h;                             // :239 unusedCapacity
        if (sw <= C || rw_q <= ds) gets = minF(rw_q, avail);  // :245
        else loop1 = true;
      } else {
        const long long cnt = count - old_s + rs_q;  // :115
        avail = C - sh + old_h;                      // :120
        eq = C / (double)cnt;                        // :123
        ds = eq * (double)rs_q;                      // :126
        if (rw_q <= ds) gets = minF(rw_q, avail);    // :131
        else loop1 = true;
      }
    }
    if (__any(loop1)) {
      // store.Map over the rows in row order (absent rows are not in the map)
      const int sl = live ? s : ~s;  // subclients + live bit (s >= 0)
      double x = 0.0, y = 0.0;
      long long wx = rs_q;  // FairShare wantExtra starts at the request's subclients (:148)
      for (int j = 0; j < K; ++j) {
        const double wj = shfl_d(w, src(j));
        const int sj = shfl_i(sl, src(j));
        if (!loop1 || sj < 0) continue;
        if (ps) {  // with server q's own request values for its row (:259-279)
          const double wv = (j == q) ? rw_q : wj;
          const int sv = (j == q) ? rs_q : sj;
          const double esp = eq * (double)sv;  // :273
          if (wv < esp)
            x += esp - wv;  // :275
          else
            y += wv - esp;  // :277
        } else if (j != q) {  // FairShare round 1, the requesting server skipped (:156-171)
          const double d = (double)sj * eq;  // :160
          if (wj < d)
            x += d - wj;  // :164
          else if (wj > d)
            wx += sj;  // :168
        }
      }
      bool loop2 = false;
      double dE = 0.0, T = 0.0;
      if (loop1) {
        if (ps) {
          gets = minF(ds + (rw_q - ds) * (x / y), avail);  // :283,290
        } else {
          dE = (x / (double)wx) * (double)rs_q;  // :175
          if (rw_q < ds + dE) gets = minF(rw_q, avail);  // :179
          else {
            T = dE + ds;  // :197 deservedExtra + deservedShare
            loop2 = true;
          }
        }
      }
      if (__any(loop2)) {
        double ee = 0.0;
        long long wee = rs_q;  // :189
        for (int j = 0; j < K; ++j) {
          const double wj = shfl_d(w, src(j));
          const int sj = shfl_i(sl, src(j));
          if (!loop2 || sj < 0 || j == q) continue;
          if (!(wj > (double)sj * eq)) continue;  // wantExtraClients (:165-169)
          if (wj < T)
            ee += T - wj;  // :197-198
          else if (wj > T)
            wee += sj;  // :199-200
        }
        if (loop2) gets = minF(ds + dE + (ee / (double)wee) * (double)rs_q, avail);  // :203-204
      }
    }
    // Assign (store.go:153-167): the running sums, and server q's row
    if (rq_q) {
      sh += gets - old_h;
      sw += rw_q - old_w;
      count += rs_q - old_s;
      if (g0 == q) {  // this lane is row q
        h = gets;
        w = rw_q;
        s = rs_q;
        live = true;
        my_gets = gets;
      }
    }
  }

  // the round's rows: the requests' leases, and the rows this round's Clean released
  const int64_t exp_new = rs_cfg.exp_out;
  if (valid) {
    if (req) {  // the root store is written in place (out_* alias its columns)
      p.out_gets[row] = my_gets;
      p.out_wants[row] = rw;
      p.out_sub[row] = (int32_t)((uint32_t)rs | kSubExplicit);
      p.out_expiry[row] = exp_new;
    } else if (expired) {
      p.out_gets[row] = 0.0;
      p.out_wants[row] = 0.0;
      p.out_sub[row] = (int32_t)kSubReleased;
      p.out_expiry[row] = kReleased;
    }
  }
  if (valid && g0 == 0) {  // the resource's first lane
    ResAgg a;
    a.count = count;
    a.sum_has = sh;
    a.sum_wants = sw;
    a.follow_exp = rs_cfg.follow_exp;
    p.res[rr] = a;
    p.expl[rr] = 1;  // the rows this tick writes carry explicit expiries
  }

  // this server's new template for the resource (server.go:279-313)
  if (mine) {
    ResCfg* c = ha.leaf_cfg + li;
    ResCold* cc = ha.leaf_cold + li;
    if (flags != 0u) {  // rejected: the templates stay (a staged slot takes a copy)
      if (ha.leaf_prev_cfg != ha.leaf_cfg) {
        *c = ha.leaf_prev_cfg[li];
        *cc = ha.leaf_prev_cold[li];
      }
    } else if (req) {
      const int64_t sec = exp_new >= 0 ? exp_new / kNs : -((-exp_new + kNs - 1) / kNs);  // time.Unix(sec, 0)
      ResCfg t;
      t.capacity = my_gets;               // :293
      t.learning_end_ns = learn;
      t.parent_expiry_ns = sec * kNs;     // :287-288
      // :295 Algorithm, from the config loaded up front (no reload after the stores above)
      t.lease_len_s = (int32_t)((exp_new - p.now) / kNs);
      t.kind = rs_cfg.kind;
      *c = t;
      ResCold tc;
      tc.safe_capacity = __builtin_isnan(rcc.safe_capacity) ? 0.0 : rcc.safe_capacity;  // :294, :894
      tc.refresh_s = rcc.refresh_s;
      tc.pad = 0;
      *cc = tc;
    } else {  // the "*" default template (server.go:53-63, :305)
      ResCfg t;
      t.capacity = 0.0;
      t.learning_end_ns = learn;
      t.parent_expiry_ns = INT64_MAX;  // expiryTimes has no entry: nil
      t.lease_len_s = 20;
      t.kind = 3;
      *c = t;
      ResCold tc;
      tc.safe_capacity = 0.0;
      tc.refresh_s = 1;
      tc.pad = 0;
      *cc = tc;
    }
  }
}

// --------------------------------------------------------------------------
// host-side launchers (called by dm_runtime.cpp)
// --------------------------------------------------------------------------
hipError_t launch_tile_small(const DevParams& p, const Tile* tiles, const TileEntry* list, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_tile_small<<<n, 256, 0, st>>>(p, tiles, list);
  return hipGetLastError();
}

// the workgroup bins (3-6) in their one-kernel form; the sub-wave bins run in k_subs
hipError_t launch_bin(int bin, const DevParams& p, WorkItem* segs, int n, int32_t* glist, int32_t* gcount,
                      hipStream_t st) {
  if (n <= 0) return hipSuccess;
  switch (bin) {
    case 3: k_block<128, 4><<<n, 128, 0, st>>>(p, segs, n, glist, gcount); break;
    case 4: k_block<128, 8><<<n, 128, 0, st>>>(p, segs, n, glist, gcount); break;
    case kBin4Wave: k_block<64, 16><<<n, 64, 0, st>>>(p, segs, n, glist, gcount); break;
    case 5: k_block<256, 8><<<n, 256, 0, st>>>(p, segs, n, glist, gcount); break;
    case 6: k_block<256, 16><<<n, 256, 0, st>>>(p, segs, n, glist, gcount); break;
    case kBin6Wide: k_block<512, 8><<<n, 512, 0, st>>>(p, segs, n, glist, gcount); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_subs(const DevParams& p, const SubBins& sb, int32_t* glist, int32_t* gcount, hipStream_t st) {
  unsigned blocks = 0;
  for (int k = 0; k < kSubShapes; ++k) blocks += (unsigned)sb.blocks[k];
  if (blocks == 0) return hipSuccess;
  k_subs<<<blocks, 256, 0, st>>>(p, sb, glist, gcount);
  return hipGetLastError();
}

// The 128-thread bins (3: 128 x 4, 4: 128 x 8) split by the dense hint: the dense
// kernel over every item, then the rest kernel over what it queued (two launches,
// timed separately).
// done (optional): an event the launch itself completes (hipExtLaunchKernel's stop
// event: no marker packet of its own on the queue), for another stream to wait on
hipError_t launch_bin_dense(int bin, const DevParams& p, WorkItem* segs, int n, int32_t* queue, int32_t* qcnt, int par,
                            int32_t* glist, int32_t* gcount, int32_t* guard, hipEvent_t done, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)n);
  switch (bin) {
    case 3:
      hipExtLaunchKernelGGL(k_block_dense<128, 4>, grid, dim3(128), 0, st, nullptr, done, 0, p, segs, n, queue, qcnt,
                            par, glist, gcount, guard);
      break;
    case 4:
      hipExtLaunchKernelGGL(k_block_dense<128, 8>, grid, dim3(128), 0, st, nullptr, done, 0, p, segs, n, queue, qcnt,
                            par, glist, gcount, guard);
      break;
    case kBin4Wave:
      hipExtLaunchKernelGGL(k_block_dense<64, 16>, grid, dim3(64), 0, st, nullptr, done, 0, p, segs, n, queue, qcnt,
                            par, glist, gcount, guard);
      break;
    case 5:
      hipExtLaunchKernelGGL(k_block_dense<256, 8>, grid, dim3(256), 0, st, nullptr, done, 0, p, segs, n, queue, qcnt,
                            par, glist, gcount, guard);
      break;
    case 6:
      hipExtLaunchKernelGGL(k_block_dense<256, 16>, grid, dim3(256), 0, st, nullptr, done, 0, p, segs, n, queue, qcnt,
                            par, glist, gcount, guard);
      break;
    case kBin6Wide:
      hipExtLaunchKernelGGL(k_block_dense<512, 8>, grid, dim3(512), 0, st, nullptr, done, 0, p, segs, n, queue, qcnt,
                            par, glist, gcount, guard);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_count_undense(const WorkItem* items, int n, unsigned long long* rec, unsigned long long epoch,
                                hipStream_t st) {
  k_count_undense<<<1, 1024, 0, st>>>(items, n, rec, epoch);
  return hipGetLastError();
}

hipError_t launch_bin_rest(int bin, const DevParams& p, WorkItem* segs, int n, int32_t* queue, int32_t* qcnt, int par,
                           int32_t* host_count, int rest_grid, int32_t* glist, int32_t* gcount, hipEvent_t done,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const dim3 rg((unsigned)std::max(1, std::min(n, rest_grid)));
  switch (bin) {
    case 3:
      hipExtLaunchKernelGGL(k_block_rest<128, 4>, rg, dim3(128), 0, st, nullptr, done, 0, p, segs, queue, qcnt, par,
                            host_count, glist, gcount);
      break;
    case 4:
      hipExtLaunchKernelGGL(k_block_rest<128, 8>, rg, dim3(128), 0, st, nullptr, done, 0, p, segs, queue, qcnt, par,
                            host_count, glist, gcount);
      break;
    case kBin4Wave:
      hipExtLaunchKernelGGL(k_block_rest<64, 16>, rg, dim3(64), 0, st, nullptr, done, 0, p, segs, queue, qcnt, par,
                            host_count, glist, gcount);
      break;
    case 5:
      hipExtLaunchKernelGGL(k_block_rest<256, 8>, rg, dim3(256), 0, st, nullptr, done, 0, p, segs, queue, qcnt, par,
                            host_count, glist, gcount);
      break;
    case 6:
      hipExtLaunchKernelGGL(k_block_rest<256, 16>, rg, dim3(256), 0, st, nullptr, done, 0, p, segs, queue, qcnt, par,
                            host_count, glist, gcount);
      break;
    case kBin6Wide:
      hipExtLaunchKernelGGL(k_block_rest<512, 8>, rg, dim3(512), 0, st, nullptr, done, 0, p, segs, queue, qcnt, par,
                            host_count, glist, gcount);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_large(int phase, const DevParams& p, const Chunk* chunks, int nchunks, const LargeSeg* ls, int nls,
                        const Partials& P, int32_t* glist, int32_t* gcount, hipStream_t st) {
  if (nchunks <= 0) return hipSuccess;
  switch (phase) {
    case 5: k_large_t<<<nls, 256, 0, st>>>(p, ls, P, glist, gcount); break;
    case 6: k_large_c_het<<<nchunks, 256, 0, st>>>(p, chunks, ls, P); break;
    case 7: k_large_e<<<dim3(nls, (kHetBuckets + 3) / 4), 256, 0, st>>>(p, ls, P); break;
    case 8: k_large_map_het<<<nchunks, 256, 0, st>>>(p, chunks, ls, P); break;
    case 0: k_large_a<<<nchunks, 256, 0, st>>>(p, chunks, P); break;
    case 1: k_large_b<<<P.b_first ? nls : nchunks, 256, 0, st>>>(p, chunks, ls, P); break;
    case 2: k_large_c<<<nchunks, 256, 0, st>>>(p, chunks, ls, P); break;
    case 3: k_large_map<<<nchunks, 256, 0, st>>>(p, chunks, ls, P, glist, gcount); break;
    case 4: k_large_fin<<<nls, 256, 0, st>>>(p, ls, P, glist, gcount); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_large_spec(int phase, const DevParams& p, const Chunk* chunks, int nchunks, const LargeSeg* ls,
                             const Partials& P, const SpecArgs& S, int redo_grid, int32_t* glist, int32_t* gcount,
                             hipStream_t st) {
  if (nchunks <= 0) return hipSuccess;
  if (phase == 0)
    k_large_spec<<<nchunks, 256, 0, st>>>(p, chunks, ls, P, S);
  else if (phase == 1)
    k_large_redo_team<false><<<redo_grid, 256, 0, st>>>(p, chunks, ls, P, S, glist, gcount);
  else
    k_large_redo_team<true><<<redo_grid, 256, 0, st>>>(p, chunks, ls, P, S, glist, gcount);
  return hipGetLastError();
}

// Workgroups of the redo's full build that one CU holds at once (the full build's grid:
// up to 3/4 of what the GPU holds, dm_runtime.cpp).
int redo_blocks_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_large_redo_team<false>, 256, 0) != hipSuccess) return 1;
  return n > 0 ? n : 1;
}

hipError_t launch_general(const DevParams& p, const int32_t* glist, const int32_t* gcount, int blocks,
                          hipStream_t st) {
  if (blocks <= 0) return hipSuccess;
  k_general<<<blocks, 256, 0, st>>>(p, glist, gcount);
  return hipGetLastError();
}

hipError_t launch_upsert(int64_t n, const int64_t* rows, const double* has, const double* wants, const int64_t* sub,
                         const int32_t* sub32, const int64_t* expiry, const ResCfg* cfg, int64_t now,
                         const RowIndex& ix, double* s_has, double* s_wants, int32_t* s_sub, int64_t* s_exp,
                         ResAgg* agg, uint8_t* expl, const uint32_t* flags, const DenseUpd& du, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_upsert<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, has, wants, sub, sub32, expiry, cfg, now, ix, s_has,
                                                        s_wants, s_sub, s_exp, agg, expl, flags, du);
  return hipGetLastError();
}

hipError_t launch_release(int64_t n, const int64_t* rows, const RowIndex& ix, double* s_has, double* s_wants,
                          int32_t* s_sub, int64_t* s_exp, ResAgg* agg, uint8_t* expl, const uint32_t* flags,
                          const DenseUpd& du, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_release<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, ix, s_has, s_wants, s_sub, s_exp, agg, expl, flags,
                                                         du);
  return hipGetLastError();
}

hipError_t launch_update_wants(int64_t n, const int64_t* rows, const double* wants, const RowIndex& ix,
                               const int32_t* s_sub, double* s_wants, ResAgg* agg, const uint32_t* flags,
                               hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_update_wants<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, wants, ix, s_sub, s_wants, agg, flags);
  return hipGetLastError();
}

hipError_t launch_resolve_rows(int64_t n, const int64_t* rows, int64_t off, const int32_t* sub, const int64_t* expiry,
                               const RowIndex& ix, const ResAgg* agg, int64_t* out_exp, int64_t* out_sub,
                               hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_resolve_rows<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, off, sub, expiry, ix, agg, out_exp, out_sub);
  return hipGetLastError();
}

hipError_t launch_gather_leases(int64_t n, const int64_t* rows, const double* gets, const int64_t* expiry,
                               double* out_gets, int64_t* out_exp, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_gather_leases<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, gets, expiry, out_gets, out_exp);
  return hipGetLastError();
}

hipError_t launch_check_rows(int64_t n, const int64_t* rows, int64_t N, uint32_t* bitmap, const double* wants,
                             const int64_t* sub, const int32_t* sub32, uint32_t* flags, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_check_rows<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, N, bitmap, wants, sub, sub32, flags);
  return hipGetLastError();
}

hipError_t launch_clear_rows(int64_t n, const int64_t* rows, int64_t N, uint32_t* bitmap, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_clear_rows<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, rows, N, bitmap);
  return hipGetLastError();
}

hipError_t launch_publish(int64_t R, const ResAgg* agg, void* dst, uint32_t* sync, hipStream_t st) {
  const int nb = (int)std::min<int64_t>(64, std::max<int64_t>(1, (R + 255) / 256));
  k_publish<<<(unsigned)nb, 256, 0, st>>>(R, agg, (double2*)dst, sync, nb);
  return hipGetLastError();
}

hipError_t launch_update_wants_mask(int64_t nwords, const uint64_t* mask, int64_t first_row, int64_t N,
                                    int64_t n_values, const double* wants, int64_t* block_sums, int32_t* word_pre,
                                    const RowIndex& ix, const int32_t* s_sub, double* s_wants, ResAgg* agg,
                                    uint32_t* flags, hipStream_t st, int phase, int64_t vlo, int64_t vhi) {
  if (nwords <= 0) return hipSuccess;
  const int64_t nb = (nwords + 255) / 256;
  if (phase != 1) {  // the mask's counts and value offsets (the mask alone)
    k_mask_count<<<(unsigned)nb, 256, 0, st>>>(nwords, mask, first_row, N, block_sums, word_pre, flags);
    k_mask_scan<<<1, 1024, 0, st>>>(nb, block_sums, n_values, flags);
  }
  if (phase != 0) {  // the rows whose values [vlo, vhi) have landed
    const int64_t waves = (nwords + kMaskWords - 1) / kMaskWords;
    k_mask_apply<<<(unsigned)((waves + 3) / 4), 256, 0, st>>>(nwords, mask, first_row, block_sums, word_pre, wants, ix,
                                                              s_sub, s_wants, agg, flags, vlo, vhi);
  }
  return hipGetLastError();
}

hipError_t launch_carry_reject(const uint32_t* from, uint32_t* to, hipStream_t st) {
  k_carry_reject<<<1, 1, 0, st>>>(from, to);
  return hipGetLastError();
}

hipError_t launch_hier_tick(const DevParams& p, const HierArgs& ha, hipStream_t st) {
  if (ha.R <= 0) return hipSuccess;
  int P = 1;
  while (P < ha.K) P <<= 1;
  const int64_t per = 64 / P;
  // at least one workgroup: block 0 also writes the round's per-server flags
  const int64_t waves = std::max<int64_t>(1, (ha.r_hi - ha.r_lo + per - 1) / per);
  k_hier_tick<<<(unsigned)((waves + 3) / 4), 256, 0, st>>>(p, ha);
  return hipGetLastError();
}

}  // namespace dm

