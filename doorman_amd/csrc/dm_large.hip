// dm_large.hip — large resources (n > kLargeMin rows) in one launch.
//
// A large resource is split into chunks of G*kFR rows, one workgroup each.  The
// per-resource totals of algorithm.go (Clean's released sums, store.go:169-181;
// FairShare round 1 extra/wantExtra, :156-171; round 2 extraExtra/wantExtraExtra
// at the threshold T, :188-204; ProportionalShare extraCapacity/extraNeed,
// :259-279) need every row of the resource before any lease can be written.  The
// five-launch chain (dm_kernels.hip, k_large_*) re-reads the rows for each of
// them; here every chunk loads its rows into VGPRs ONCE and the chunks of one
// resource exchange their partial sums inside the launch:
//
//   chunk: rows -> partial -> write-through store -> arrive (agent atomic add)
//   the last arriver (told by the value its add returned) reduces the resource's
//   partials in a fixed order, stores the totals write-through and sets the
//   phase's flag to the launch epoch; every other chunk polls that flag (one lane,
//   relaxed agent loads, s_sleep) and loads the totals.
//
// Hand-off form: MI355X_MICROARCH.md "Valid forms", first table row — payload and
// totals stored with 8-B agent-scope atomic stores (write-through, no release
// fence, so the chunks' dirty output lines are never written back early), every
// storing wave drains with s_waitcnt vmcnt(0) before its arrive/flag, every load of
// handed-off bytes is an agent-scope atomic load (L1 bypassed), no acquire fence.
// All chunks of a resource use the last arriver's totals (one fixed tree), so the
// results are deterministic; they match the chain's within rounding (different
// chunking and reduction trees), both against the oracle at the survey's bar.
//
// Co-residency: a chunk waits only for chunks of its own resource.  Chunks take a
// ticket from a dispenser, so they start in resource order; a resource's chunks are
// then all resident or finished once its last chunk has a ticket, which holds as long
// as no resource has more chunks than the device keeps resident.  The planner uses
// this kernel only when every large resource has at most half that many chunks
// and at most G (one record per thread of the last arriver; dm_runtime.cpp); every
// wait is bounded and a wait that gives up sets a host-visible error word (the tick
// then reports DM_E_HIP) instead of hanging.  A chunk whose wait gave up writes
// nothing after it, but other chunks may already have written their leases, so
// after such a writeback tick the host treats the store as lost until it is
// loaded again (dm_runtime.cpp, check_fused).
#include <hip/hip_runtime.h>

#include "dm_records.h"

namespace dm {

constexpr int kFR = kFusedRows;  // rows per thread held in VGPRs

// Last arriver: the resource's totals from every chunk's record.  Thread t loads
// record t (a resource has at most G chunks here: the planner's bound), so every
// load is in flight at once; the records are combined by group_reduce's fixed tree.
template <int G>
__device__ __forceinline__ AggA all_reduce_a(const DevParams& p, const FusedState& F, const LargeSeg& L, Lds<G>& lds) {
  const int c = L.chunk_begin + (int)threadIdx.x;
  const AggA x = c < L.chunk_end ? load_a(F.part + (size_t)c * kFusedWords) : zeroA();
  AggA a = group_reduce<G>(x, OpA(), lds.a);
  if (p.recompute) a.all = group_reduce<G>(x.all, OpR(), lds.r);
  return a;
}
template <int G>
__device__ __forceinline__ AggB all_reduce_b(const FusedState& F, const LargeSeg& L, Lds<G>& lds) {
  const int c = L.chunk_begin + (int)threadIdx.x;
  const AggB x = c < L.chunk_end ? load_b(F.part + (size_t)c * kFusedWords) : AggB{0.0, 0.0, 0};
  return group_reduce<G>(x, OpB(), lds.b);
}
template <int G>
__device__ __forceinline__ AggC all_reduce_c(const FusedState& F, const LargeSeg& L, Lds<G>& lds) {
  const int c = L.chunk_begin + (int)threadIdx.x;
  const AggC x = c < L.chunk_end ? load_c(F.part + (size_t)c * kFusedWords) : AggC{0.0, 0};
  return group_reduce<G>(x, OpC(), lds.c);
}

// One exchange of a phase: lane 0 has stored this chunk's record; returns (to every
// thread) after the resource's totals words [w0, w1) are in xt.  The last arriver
// reduces and publishes them (reduce(), then its flag); the others poll the flag.
// Returns false (uniformly) when the poll gave up: the chunk must then write
// nothing more (the host reports the tick as failed and the store as unusable).
template <int G, typename Reduce>
__device__ __forceinline__ bool exchange(uint32_t* ctr, uint32_t* flags, int ci, const FusedState& F, int nch,
                                         uint64_t* trec, uint64_t* xt, uint32_t* xl, int w0, int w1, Reduce reduce) {
  if (threadIdx.x < 64) {
    const bool last = arrive_last(ctr, nch);
    if (threadIdx.x == 0) *xl = last ? 1u : 0u;
  }
  __syncthreads();
  if (*xl) {
    reduce();  // every thread; lane 0 stores the totals words write-through
    if (threadIdx.x < 64) publish_flag(flags, F.epoch);
  } else if (threadIdx.x == 0) {
    if (!wait_flag(flags + (ci % kFusedFlagCopies) * 32, F.epoch, F.spin_limit, F.err)) *xl = 2u;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: loads stay below the poll
  }
  if (threadIdx.x == 0)
    for (int i = w0; i < w1; ++i) xt[i] = ld_wt(trec + i);
  __syncthreads();
  return *xl != 2u;
}

template <int G>
__global__ __launch_bounds__(G, 1024 / G) void k_large_fused(DevParams p, const Chunk* __restrict__ chunks,
                                                   const LargeSeg* __restrict__ ls, FusedState F,
                                                   int32_t* general_list, int32_t* general_count) {
  __shared__ Lds<G> lds;
  __shared__ uint32_t xw;       // the ticket
  __shared__ uint32_t xl[4];    // per phase: this workgroup arrived last
  __shared__ uint64_t xt[16];   // a phase's totals, broadcast to the workgroup (totals-record layout)
  const int t = threadIdx.x;
  if (t == 0) {
    const uint32_t tk = __hip_atomic_fetch_add((gu32*)F.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (uint32_t)F.nchunks - 1) __hip_atomic_store((gu32*)F.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    xw = tk;
  }
  __syncthreads();
  const int ci = __builtin_amdgcn_readfirstlane((int)xw);  // uniform: the chunk record and row bases stay scalar
  const Chunk ch = chunks[ci];
  const double* __restrict__ wb = p.wants + ch.row0;
  const double* __restrict__ hb = p.has + ch.row0;
  const int32_t* __restrict__ sb = p.sub + ch.row0;
  const int64_t* __restrict__ eb = p.expiry + ch.row0;
  double w[kFR], h[kFR];
  int s[kFR], sr[kFR];  // subclients, and the raw words (expiry encoding, dm_device.h)
  unsigned valid = 0, live = 0;
  const Res rs = load_res(p, ch.seg);
  {
#pragma unroll
    for (int k = 0; k < kFR; ++k) {  // every load issued before the first use (dm_kernels.hip, load_chunk)
      const int i = k * G + t;
      const unsigned u = (unsigned)(i < ch.nrows ? i : ch.nrows - 1);
      w[k] = wb[u];
      h[k] = hb[u];
      sr[k] = sb[u];
      if (k == kFR / 2 - 1) __builtin_amdgcn_s_waitcnt(0x0F70);  // two round trips of half the rows
    }
    int64_t e[kFR];
#pragma unroll
    for (int k = 0; k < kFR; ++k) e[k] = rs.follow_exp;
    if (any_explicit(rs)) {  // the resource's flag (dm_kernels.hip, group_segment)
#pragma unroll
      for (int k = 0; k < kFR; ++k) {
        const int i = k * G + t;
        const int64_t x = eb[(unsigned)(i < ch.nrows ? i : ch.nrows - 1)];
        if (sub_explicit(sr[k])) e[k] = x;
      }
    }
#pragma unroll
    for (int k = 0; k < kFR; ++k) {
      const unsigned vk = (k * G + t < ch.nrows) ? 1u : 0u;
      valid |= vk << k;
      if (sub_released(sr[k])) e[k] = kReleased;
      live |= (vk & (p.now > e[k] ? 0u : 1u)) << k;  // store.go:174
      s[k] = sub_value(sr[k]);
    }
  }
  const LargeSeg L = ls[ch.lseg];
  const int nch = L.chunk_end - L.chunk_begin;
  uint32_t* sy = F.sync + (size_t)ch.lseg * kFusedSync;  // arrive[0..3]; flags of phase k at sy + flag_at(k)
  uint64_t* prec = F.part + (size_t)ci * kFusedWords;
  uint64_t* trec = F.tot + (size_t)ch.lseg * kFusedWords;

  // ---- pass A (Clean sums) + speculative pass B (equalShare from the running Count) ----
  const bool need_tot = !rs.learning && rs.kind >= 2;  // ProportionalShare / FairShare
  const bool spec = !p.recompute && need_tot;
  AggA a = zeroA();
  AggB b{0.0, 0.0, 0};
  {
    const double eq0 = rs.C / (double)rs.agg_count;
#pragma unroll
    for (int k = 0; k < kFR; ++k) {
      if (!(valid >> k & 1)) continue;
      const bool lv = live >> k & 1;
      if (!lv) {
        a.cnt += s[k];
        a.h += h[k];
        a.w += w[k];
      }
      if (p.recompute) {
        a.all.cnt += s[k];
        a.all.h += h[k];
        a.all.w += w[k];
      }
      if (lv) {
        a.smin = s[k] < a.smin ? s[k] : a.smin;
        a.smax = s[k] > a.smax ? s[k] : a.smax;
        a.nan |= __builtin_isnan(w[k]) ? 1 : 0;
        if (spec) {
          if (rs.kind == 2) {
            const double ex = eq0 * (double)s[k];  // algorithm.go:273
            if (w[k] < ex)
              b.x += ex - w[k];  // :275
            else
              b.y += w[k] - ex;  // :277
          } else {
            const double d = (double)s[k] * eq0;  // :160
            if (w[k] < d)
              b.x += d - w[k];  // :164
            else if (w[k] > d)
              b.i += s[k];  // :168
          }
        }
      }
    }
    const AggR all_part = a.all;
    a = group_reduce<G>(a, OpA(), lds.a);
    if (p.recompute) a.all = group_reduce<G>(all_part, OpR(), lds.r);
    if (spec) b = group_reduce<G>(b, OpB(), lds.b);
  }
  if (t == 0) {
    store_a(prec, a);
    if (spec) store_b(prec, b);
  }

  SegState st;
  AggB tb{0.0, 0.0, 0};
  if (need_tot) {
    if (!exchange<G>(sy + 0, sy + flag_at(0), ci, F, nch, trec, xt, &xl[0], 0, 11, [&] {  // pass-A (and speculative B) totals
          const AggA ta = all_reduce_a<G>(p, F, L, lds);
          const AggB sb2 = spec ? all_reduce_b<G>(F, L, lds) : AggB{0.0, 0.0, 0};
          if (t == 0) {
            store_a(trec, ta);
            store_b(trec, sb2);
            if (seg_state_of(p, ch.seg, ta).general) general_list[atomicAdd(general_count, 1)] = ch.seg;  // k_general
          }
        }))
      return;
    st = seg_state_of(p, ch.seg, xt_a(xt));
    tb = AggB{dbl(xt[8]), dbl(xt[9]), (long long)xt[10]};
    if (st.general) return;  // heterogeneous-subclient FairShare: k_general decides the resource
  }
  const double C = rs.C;
  const double eq = need_tot ? C / (double)st.cl.count : 0.0;

  // ---- pass B again when Clean released subclients (or recompute mode) ----
  if (need_tot && !(spec && st.a.cnt == 0)) {
    AggB bb{0.0, 0.0, 0};
#pragma unroll
    for (int k = 0; k < kFR; ++k) {
      if (!(live >> k & 1)) continue;
      if (rs.kind == 2) {
        const double ex = eq * (double)s[k];
        if (w[k] < ex)
          bb.x += ex - w[k];
        else
          bb.y += w[k] - ex;
      } else {
        const double d = (double)s[k] * eq;
        if (w[k] < d)
          bb.x += d - w[k];
        else if (w[k] > d)
          bb.i += s[k];
      }
    }
    bb = group_reduce<G>(bb, OpB(), lds.b);
    if (t == 0) store_b(prec, bb);
    if (!exchange<G>(sy + 1, sy + flag_at(1), ci, F, nch, trec, xt, &xl[1], 8, 11, [&] {
          const AggB x = all_reduce_b<G>(F, L, lds);
          if (t == 0) store_b(trec, x);
        }))
      return;
    tb = AggB{dbl(xt[8]), dbl(xt[9]), (long long)xt[10]};
  }

  // ---- pass C: FairShare round 2 at the resource's one threshold (uniform subclients) ----
  const bool fs = need_tot && rs.kind == 3;
  AggC tc{0.0, 0};
  if (fs) {
    const double s0 = (double)st.a.smin;
    const double Tu = (tb.x / (double)tb.i) * s0 + eq * s0;  // :175,197 (as k_large_c)
    AggC c{0.0, 0};
#pragma unroll
    for (int k = 0; k < kFR; ++k) {
      if (!(live >> k & 1)) continue;
      if (!(w[k] > (double)s[k] * eq)) continue;  // wantExtraClients (:165-169)
      if (w[k] < Tu)
        c.ee += Tu - w[k];  // :197-198
      else if (w[k] > Tu)
        c.sgt += s[k];  // :199-200
    }
    c = group_reduce<G>(c, OpC(), lds.c);
    if (t == 0) store_c(prec, c);
    if (!exchange<G>(sy + 2, sy + flag_at(2), ci, F, nch, trec, xt, &xl[2], 11, 13, [&] {
          const AggC x = all_reduce_c<G>(F, L, lds);
          if (t == 0) store_c(trec, x);
        }))
      return;
    tc = AggC{dbl(xt[11]), (long long)xt[12]};
  }

  // ---- map: decide and write every lease (store.go:153-167 Assign) ----
  const FsU fu = fs ? make_fsu(eq, st.a.smin, tb.x, tb.i, tc) : FsU{0.0, 0.0, 0.0, 0.0, 0.0};
  SumD delta{0.0};
#pragma unroll
  for (int k = 0; k < kFR; ++k) {
    if (!(valid >> k & 1)) continue;
    const unsigned u = (unsigned)(k * G + t);
    if (!(live >> k & 1)) {  // released by Clean: no lease
      put_released(p, ch.row0, u, sr[k]);
      continue;
    }
    double g;
    if (rs.learning) {
      g = h[k];  // Learn (algorithm.go:297-302)
    } else if (rs.kind == 0) {
      g = w[k];  // NoAlgorithm
    } else if (rs.kind == 1) {
      g = minF(C, w[k]);  // Static
    } else if (rs.kind == 2) {
      const double epc = eq * (double)s[k];             // :233
      const double unused = C - st.cl.sum_has + h[k];  // :239
      g = (st.cl.sum_wants <= C || w[k] <= epc) ? minF(w[k], unused)                            // :245
                                                 : minF(epc + (w[k] - epc) * (tb.x / tb.y), unused);  // :283
    } else {
      g = fs_uniform_row(w[k], h[k], C, st.cl.sum_has, fu);
    }
    put_live(p, ch.row0, u, g, rs, sr[k]);
    delta.v += g - h[k];
  }
  delta = group_reduce<G>(delta, OpSumD(), lds.d);
  // ---- the resource's record: the last chunk to finish writes it (no one waits) ----
  if (t == 0) st_wt(prec + 13, bits(delta.v));
  if (t < 64) {
    const bool last = arrive_last(sy + 3, nch);
    if (t == 0) xl[3] = last ? 1u : 0u;
  }
  __syncthreads();
  if (!xl[3]) return;
  const int q = L.chunk_begin + t;
  const SumD d = group_reduce<G>(SumD{q < L.chunk_end ? dbl(ld_wt(F.part + (size_t)q * kFusedWords + 13)) : 0.0},
                                 OpSumD(), lds.d);
  if (!need_tot) st = seg_state_of(p, ch.seg, all_reduce_a<G>(p, F, L, lds));  // no pass-A exchange ran
  if (t == 0) write_resource(p, ch.seg, st.rs, st.cl, d.v);
}

hipError_t launch_large_fused(int G, const DevParams& p, const Chunk* chunks, const LargeSeg* ls, const FusedState& F,
                              int32_t* glist, int32_t* gcount, hipStream_t st) {
  if (F.nchunks <= 0) return hipSuccess;
  switch (G) {
    case 256: k_large_fused<256><<<F.nchunks, 256, 0, st>>>(p, chunks, ls, F, glist, gcount); break;
    case 512: k_large_fused<512><<<F.nchunks, 512, 0, st>>>(p, chunks, ls, F, glist, gcount); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Workgroups of k_large_fused<G> one CU keeps resident (the co-residency bound).
hipError_t large_fused_occupancy(int G, int* blocks_per_cu) {
  switch (G) {
    case 256: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_large_fused<256>, 256, 0);
    case 512: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_large_fused<512>, 512, 0);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dm
