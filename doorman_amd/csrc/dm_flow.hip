// dm_flow.hip — large resources (n > kLargeMin rows) in ONE persistent launch.
//
// The chain (dm_kernels.hip, k_large_{a,b,c,map,fin}) runs the per-resource totals
// of algorithm.go as stream-ordered launches: Clean's released sums + a speculative
// round 1 (store.go:169-181, algorithm.go:156-171 / :259-279), round 1 again where
// Clean released subclients, FairShare round 2 (:188-204), the map (store.go:153-167
// Assign), the records.  Each launch boundary drains the GPU of the class's work
// and every chunk re-reduces its resource's partials (O(chunks^2) per resource).
//
// Here the same phases are tasks of one launch.  The host lists them so that every
// task comes after the tasks it needs (its resource's earlier phases); a fixed grid
// of workgroups takes tasks in list order from a ticket counter (the next ticket is
// fetched while the current task runs).  Per resource and phase the chunks arrive
// at a counter; the last arriver reduces the chunk records in a fixed order, stores
// the totals and sets the phase's flag (dm_records.h: write-through records, agent
// atomics, replicated flags); a later phase's task polls the flag.  Deadlock-free
// with any number of resident workgroups: a waiting task waits only for tasks with
// smaller tickets, and every ticket handed out belongs to a running workgroup (by
// induction the smallest unfinished ticket can always proceed).  Every wait is
// bounded anyway; a wait that gives up sets the host-mapped error word and the
// workgroup stops (the host then reports the tick failed, as for the fused path).
//
// The list interleaves resources' phases (pass A of later resources between the
// round-2 and map tasks of earlier ones), so a chunk's rows are
// re-read a short while after pass A read them, while they are likely still in the
// Infinity Cache.  Results are deterministic (fixed reduction trees) and agree with
// the chain's within rounding; both are tested against the oracle.
#include <hip/hip_runtime.h>

#include "dm_records.h"

namespace dm {

constexpr int kFlR = kChunkRows / 256;  // rows per thread

struct FlRows {
  double w[kFlR], h[kFlR];
  int s[kFlR];
  unsigned valid, live, expl, rel;
};

struct FlLds {
  Lds<256> lds;
  uint64_t xt[16];  // a resource's totals words, broadcast
  uint32_t ok;      // a wait's outcome / this workgroup arrived last
  uint32_t next;    // the next ticket
};

// threadIdx.x as a value the compiler cannot hoist out of the task loop: otherwise
// every per-row byte offset of every task is computed once before the loop and held
// in VGPRs across it (k_large_flow 137 -> the largest task's own count)
__device__ __forceinline__ int fl_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ uint32_t* fl_sync(const FlowState& F, int lseg) { return F.sync + (size_t)lseg * kFusedSync; }
__device__ __forceinline__ uint64_t* fl_part(const FlowState& F, int c) { return F.part + (size_t)c * kFusedWords; }
__device__ __forceinline__ uint64_t* fl_tot(const FlowState& F, int lseg) { return F.tot + (size_t)lseg * kFusedWords; }

// Thread 0 polls phase `ph`'s flag of resource lseg (replica by chunk), then loads the
// totals words [w0, w1) into S.xt; returns to every thread whether the wait succeeded.
__device__ __forceinline__ bool fl_wait(const FlowState& F, int lseg, int ph, int rep, int w0, int w1, FlLds& S) {
  __syncthreads();  // S.xt / S.ok of an earlier wait are read
  if (threadIdx.x == 0) {
    const bool ok = wait_flag(fl_sync(F, lseg) + flag_at(ph) + (rep % kFusedFlagCopies) * 32, F.epoch,
                              F.spin_limit, F.err);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: the loads stay below the poll
    if (ok)
      for (int i = w0; i < w1; ++i) S.xt[i] = ld_wt(fl_tot(F, lseg) + i);
    S.ok = ok ? 1u : 0u;
  }
  __syncthreads();
  return S.ok != 0;
}

// After thread 0 stored this chunk's record (and every wave drained its own
// write-through stores): arrive at counter k of resource lseg; true (uniform) when
// this workgroup arrived last.
// every_wave: every wave stored bytes the later tasks read (pass A's row masks);
// otherwise only thread 0 did, and arrive_last drains its wave.
__device__ __forceinline__ bool fl_arrive(const FlowState& F, int lseg, int k, int n, FlLds& S,
                                          bool every_wave = false) {
  if (every_wave) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's row masks landed
  __syncthreads();
  if (threadIdx.x < 64) {
    const bool last = arrive_last(fl_sync(F, lseg) + k, n);
    if (threadIdx.x == 0) S.ok = last ? 1u : 0u;
  }
  __syncthreads();
  return S.ok != 0;
}

// rows of chunk ch: wants, and subclients when with_sub (loads issued before any is
// consumed; lanes past the chunk re-read its last row)
__device__ __forceinline__ void fl_issue(const DevParams& p, const Chunk& ch, FlRows& r, int* sr, bool with_sub,
                                         bool with_has, int t) {
  const double* __restrict__ wb = p.wants + ch.row0;
  const double* __restrict__ hb = p.has + ch.row0;
  const int32_t* __restrict__ sb = p.sub + ch.row0;
#pragma unroll
  for (int k = 0; k < kFlR; ++k) {
    const int i = k * 256 + t;
    const unsigned u = (unsigned)(i < ch.nrows ? i : ch.nrows - 1);
    r.w[k] = *col_at(wb, u);
    r.h[k] = with_has ? *col_at(hb, u) : 0.0;
    sr[k] = with_sub ? *col_at(sb, u) : 0;
  }
}

// the row masks pass A left for chunk c (written in this launch: agent-scope load)
__device__ __forceinline__ void fl_masks(const FlowState& F, int c, const Chunk& ch, FlRows& r, const int* sr,
                                         bool with_sub, int t) {
  const uint32_t m = (uint32_t)ld_wt((const int32_t*)F.live + (size_t)c * 256 + t);
  r.live = m & 0xFFu;
  r.expl = (m >> 8) & 0xFFu;
  r.rel = (m >> 16) & 0xFFu;
  r.valid = 0;
#pragma unroll
  for (int k = 0; k < kFlR; ++k) {
    const bool v = k * 256 + t < ch.nrows;
    r.valid |= (v ? 1u : 0u) << k;
    r.s[k] = (v && with_sub) ? sub_value(sr[k]) : 0;
    if (!v) {
      r.w[k] = 0.0;
      r.h[k] = 0.0;
    }
  }
}

// ---- pass A: Clean's sums + speculative round 1 (as k_large_a) ----
__device__ bool fl_task_a(const DevParams& p, const FlowState& F, int c, FlLds& S, int32_t* glist,
                          int32_t* gcount) {
  const int t = fl_tid();
  const Chunk ch = F.chunks[c];
  const Res rs = load_res(p, ch.seg);
  FlRows rw;
  int sr[kFlR];
  {
    const double* __restrict__ wb = p.wants + ch.row0;
    const double* __restrict__ hb = p.has + ch.row0;
    const int32_t* __restrict__ sb = p.sub + ch.row0;
    const int64_t* __restrict__ eb = p.expiry + ch.row0;
    rw.valid = rw.live = rw.expl = rw.rel = 0;
#pragma unroll
    for (int k = 0; k < kFlR; ++k) {
      const int i = k * 256 + t;
      const unsigned u = (unsigned)(i < ch.nrows ? i : ch.nrows - 1);
      rw.w[k] = *col_at(wb, u);
      sr[k] = *col_at(sb, u);
      rw.h[k] = 0.0;
    }
    int64_t e[kFlR];
#pragma unroll
    for (int k = 0; k < kFlR; ++k) e[k] = rs.follow_exp;
    if (any_explicit(rs)) {
#pragma unroll
      for (int k = 0; k < kFlR; ++k) {
        const int i = k * 256 + t;
        const int64_t x = *col_at(eb, (unsigned)(i < ch.nrows ? i : ch.nrows - 1));
        if (sub_explicit(sr[k])) e[k] = x;
      }
    }
#pragma unroll
    for (int k = 0; k < kFlR; ++k) {
      const unsigned vk = (k * 256 + t < ch.nrows) ? 1u : 0u;
      rw.valid |= vk << k;
      if (sub_released(sr[k])) e[k] = kReleased;
      rw.live |= (vk & (p.now > e[k] ? 0u : 1u)) << k;  // store.go:174 (strict After)
      rw.expl |= (sub_explicit(sr[k]) ? 1u : 0u) << k;
      rw.rel |= (sub_released(sr[k]) ? 1u : 0u) << k;
      rw.s[k] = sub_value(sr[k]);
    }
    const unsigned need_h = p.recompute ? rw.valid : (rw.valid & ~rw.live);  // has: released rows only
    if (__any(need_h != 0)) {
#pragma unroll
      for (int k = 0; k < kFlR; ++k)
        if (need_h >> k & 1) rw.h[k] = *col_at(hb, (unsigned)(k * 256 + t));
    }
  }
  st_wt((int32_t*)F.live + (size_t)c * 256 + t, (int32_t)(rw.live | rw.expl << 8 | rw.rel << 16));
  AggA a = zeroA();
  const bool spec = !p.recompute && !rs.learning && rs.kind >= 2;
  AggB b{0.0, 0.0, 0};
  const double eq0 = rs.C / (double)rs.agg_count;
#pragma unroll
  for (int k = 0; k < kFlR; ++k) {
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
      if (spec) {
        const double w = rw.w[k];
        const int sk = rw.s[k];
        if (rs.kind == 2) {
          const double e = eq0 * (double)sk;  // algorithm.go:273
          if (w < e)
            b.x += e - w;  // :275
          else
            b.y += w - e;  // :277
        } else {
          const double d = (double)sk * eq0;  // :160
          if (w < d)
            b.x += d - w;  // :164
          else if (w > d)
            b.i += sk;  // :168
        }
      }
    }
  }
  {
    const AggR all_part = a.all;
    a = group_reduce<256>(a, OpA(), S.lds.a);
    if (p.recompute) a.all = group_reduce<256>(all_part, OpR(), S.lds.r);
    if (spec) b = group_reduce<256>(b, OpB(), S.lds.b);
  }
  if (t == 0) {
    store_a(fl_part(F, c), a);
    if (spec) store_b(fl_part(F, c), b);
  }
  const LargeSeg L = F.large[ch.lseg];
  if (!fl_arrive(F, ch.lseg, 0, L.chunk_end - L.chunk_begin, S, true)) return true;
  // last arriver: the resource's pass-A (and speculative round-1) totals, fixed order
  AggA x = zeroA();
  AggR xall{0, 0.0, 0.0};
  AggB xb{0.0, 0.0, 0};
  for (int q = L.chunk_begin + t; q < L.chunk_end; q += 256) {
    const AggA y = load_a(fl_part(F, q));
    xall = OpR()(xall, y.all);
    x = OpA()(x, y);
    if (spec) xb = OpB()(xb, load_b(fl_part(F, q)));
  }
  x = group_reduce<256>(x, OpA(), S.lds.a);
  x.all = p.recompute ? group_reduce<256>(xall, OpR(), S.lds.r) : AggR{0, 0.0, 0.0};
  if (spec) xb = group_reduce<256>(xb, OpB(), S.lds.b);
  if (t == 0) {
    store_a(fl_tot(F, ch.lseg), x);
    store_b(fl_tot(F, ch.lseg), xb);
    if (seg_state_of(p, L.seg, x).general) glist[atomicAdd(gcount, 1)] = L.seg;  // k_general decides it
  }
  if (t < 64) publish_flag(fl_sync(F, ch.lseg) + flag_at(0), F.epoch);
  return true;
}

// whether round 1 must be recomputed from the rows: Clean released subclients (the
// speculative equalShare used the pre-Clean count) or the sums are rebuilt
__device__ __forceinline__ bool fl_need_b(const DevParams& p, const SegState& st) {
  return !st.rs.learning && st.rs.kind >= 2 && !st.general && (p.recompute || st.a.cnt != 0);
}

// ---- round 1 again, for up to kFlowBundle chunks of one resource (as k_large_b) ----
__device__ bool fl_task_b(const DevParams& p, const FlowState& F, int c0, FlLds& S) {
  const int t = fl_tid();
  const Chunk ch0 = F.chunks[c0];
  {
    const ResCfg cf = p.cfg[ch0.seg];
    if (cf.learning_end_ns > p.now || cf.kind < 2) return true;  // only PS / FS have a round 1
  }
  const LargeSeg L = F.large[ch0.lseg];
  if (!fl_wait(F, ch0.lseg, 0, c0, 0, 11, S)) return false;
  const SegState st = seg_state_of(p, L.seg, uniform(xt_a(S.xt)));
  if (!fl_need_b(p, st)) return true;
  const bool ps = st.rs.kind == 2;
  const double eq = st.rs.C / (double)st.cl.count;
  const int cend = min(c0 + kFlowBundle, L.chunk_end);
  for (int c = c0; c < cend; ++c) {
    const Chunk ch = F.chunks[c];
    FlRows rw;
    int sr[kFlR];
    fl_issue(p, ch, rw, sr, ps, false, t);
    fl_masks(F, c, ch, rw, sr, ps, t);
    AggB bb{0.0, 0.0, 0};
#pragma unroll
    for (int k = 0; k < kFlR; ++k) {
      if (!(rw.live >> k & 1)) continue;
      const double w = rw.w[k];
      if (ps) {
        const double e = eq * (double)rw.s[k];
        if (w < e)
          bb.x += e - w;
        else
          bb.y += w - e;
      } else {  // uniform FairShare: one count
        const int s = st.a.smin;
        const double d = (double)s * eq;
        if (w < d)
          bb.x += d - w;
        else if (w > d)
          bb.i += s;
      }
    }
    bb = group_reduce<256>(bb, OpB(), S.lds.b);
    if (t == 0) store_b(fl_part(F, c), bb);
  }
  const int nb = (L.chunk_end - L.chunk_begin + kFlowBundle - 1) / kFlowBundle;
  if (!fl_arrive(F, ch0.lseg, 1, nb, S)) return true;
  AggB xb{0.0, 0.0, 0};
  for (int q = L.chunk_begin + t; q < L.chunk_end; q += 256) xb = OpB()(xb, load_b(fl_part(F, q)));
  xb = group_reduce<256>(xb, OpB(), S.lds.b);
  if (t == 0) store_b(fl_tot(F, ch0.lseg), xb);
  if (t < 64) publish_flag(fl_sync(F, ch0.lseg) + flag_at(1), F.epoch);
  return true;
}

// ---- FairShare round 2 at the resource's one threshold (as k_large_c) ----
__device__ bool fl_task_c(const DevParams& p, const FlowState& F, int c, FlLds& S) {
  const int t = fl_tid();
  const Chunk ch = F.chunks[c];
  {
    const ResCfg cf = p.cfg[ch.seg];
    if (cf.learning_end_ns > p.now || cf.kind != 3) return true;  // only FairShare has a round 2
  }
  FlRows rw;
  int sr[kFlR];
  fl_issue(p, ch, rw, sr, false, false, t);  // rows in flight while the totals are awaited
  const LargeSeg L = F.large[ch.lseg];
  if (!fl_wait(F, ch.lseg, 0, c, 0, 11, S)) return false;
  const SegState st = seg_state_of(p, L.seg, uniform(xt_a(S.xt)));
  if (st.general || st.rs.learning || st.rs.kind != 3) return true;
  if (fl_need_b(p, st) && !fl_wait(F, ch.lseg, 1, c, 8, 11, S)) return false;
  const AggB b = uniform(xt_b(S.xt));
  fl_masks(F, c, ch, rw, sr, false, t);
  const double eq = st.rs.C / (double)st.cl.count;
  const int s0 = st.a.smin;
  const double Tu = (b.x / (double)b.i) * (double)s0 + eq * (double)s0;  // :175,197 (as k_large_c)
  AggC cc{0.0, 0};
#pragma unroll
  for (int k = 0; k < kFlR; ++k) {
    if (!(rw.live >> k & 1)) continue;
    const double w = rw.w[k];
    if (!(w > (double)s0 * eq)) continue;  // wantExtraClients (:165-169)
    if (w < Tu)
      cc.ee += Tu - w;  // :197-198
    else if (w > Tu)
      cc.sgt += s0;  // :199-200
  }
  cc = group_reduce<256>(cc, OpC(), S.lds.c);
  if (t == 0) store_c(fl_part(F, c), cc);
  if (!fl_arrive(F, ch.lseg, 2, L.chunk_end - L.chunk_begin, S)) return true;
  AggC xc{0.0, 0};
  for (int q = L.chunk_begin + t; q < L.chunk_end; q += 256) xc = OpC()(xc, load_c(fl_part(F, q)));
  xc = group_reduce<256>(xc, OpC(), S.lds.c);
  if (t == 0) store_c(fl_tot(F, ch.lseg), xc);
  if (t < 64) publish_flag(fl_sync(F, ch.lseg) + flag_at(2), F.epoch);
  return true;
}

// ---- the map: decide and write every lease (as k_large_map); the resource's last
// chunk writes its record (as k_large_fin) ----
__device__ bool fl_task_m(const DevParams& p, const FlowState& F, int c, FlLds& S) {
  const int t = fl_tid();
  const Chunk ch = F.chunks[c];
  bool ps, fs;
  {
    const ResCfg cf = p.cfg[ch.seg];
    const bool lrn = cf.learning_end_ns > p.now;
    ps = !lrn && cf.kind == 2;
    fs = !lrn && cf.kind == 3;
  }
  FlRows rw;
  int sr[kFlR];
  fl_issue(p, ch, rw, sr, ps, true, t);  // rows in flight while the totals are awaited
  const LargeSeg L = F.large[ch.lseg];
  if (!fl_wait(F, ch.lseg, 0, c, 0, 11, S)) return false;
  const SegState st = seg_state_of(p, L.seg, uniform(xt_a(S.xt)));
  if (st.general) return true;  // k_general decides the resource
  if (fl_need_b(p, st) && !fl_wait(F, ch.lseg, 1, c, 8, 11, S)) return false;
  if (fs && !fl_wait(F, ch.lseg, 2, c, 11, 13, S)) return false;
  fl_masks(F, c, ch, rw, sr, ps, t);
  // only the scalars the map needs stay live through it (the resource's state is
  // re-derived from S.xt by the last arriver): fewer SGPRs, no spills into VGPRs
  const int kind = __builtin_amdgcn_readfirstlane(st.rs.learning ? -1 : st.rs.kind);
  const double C = uniform(st.rs.C);
  const double sh = uniform(st.cl.sum_has), sw = uniform(st.cl.sum_wants);
  const double eq = uniform(C / (double)st.cl.count);
  double r_ps = 0.0;
  FsU fu{0.0, 0.0, 0.0, 0.0, 0.0};
  if (kind == 2) {
    const AggB b = uniform(xt_b(S.xt));
    r_ps = uniform(b.x / b.y);
  } else if (kind == 3) {
    const AggB b = uniform(xt_b(S.xt));
    fu = uniform(make_fsu(eq, st.a.smin, b.x, b.i, uniform(xt_c(S.xt))));
  }
  Res ro;  // put_live reads exp_out only
  ro.exp_out = uniform(st.rs.exp_out);
  SumD delta{0.0};
#pragma unroll
  for (int k = 0; k < kFlR; ++k) {
    if (!(rw.valid >> k & 1)) continue;
    const unsigned u = (unsigned)(k * 256 + t);
    const double w = rw.w[k], h = rw.h[k];
    if (!(rw.live >> k & 1)) {  // released by Clean
      put_released(p, ch.row0, u, (rw.rel >> k & 1) ? (int32_t)kSubReleased : 0);
      continue;
    }
    double g;
    if (kind < 0) {
      g = h;  // Learn (algorithm.go:297-302)
    } else if (kind == 0) {
      g = w;  // NoAlgorithm
    } else if (kind == 1) {
      g = minF(C, w);  // Static
    } else if (kind == 2) {
      const double epc = eq * (double)rw.s[k];  // :233
      const double unused = C - sh + h;         // :239
      g = (sw <= C || w <= epc) ? minF(w, unused)                      // :245
                                : minF(epc + (w - epc) * r_ps, unused);  // :283
    } else {
      g = fs_uniform_row(w, h, C, sh, fu);
    }
    put_live(p, ch.row0, u, g, ro, (rw.expl >> k & 1) ? (p.sub[ch.row0 + u] | (int32_t)kSubExplicit) : 0);
    delta.v += g - h;
  }
  delta = group_reduce<256>(delta, OpSumD(), S.lds.d);
  if (t == 0) st_wt(fl_part(F, c) + 13, bits(delta.v));
  if (!fl_arrive(F, ch.lseg, 3, L.chunk_end - L.chunk_begin, S)) return true;
  SumD d{0.0};
  for (int q = L.chunk_begin + t; q < L.chunk_end; q += 256) d.v += dbl(ld_wt(fl_part(F, q) + 13));
  d = group_reduce<256>(d, OpSumD(), S.lds.d);
  if (t == 0) {
    const SegState sf = seg_state_of(p, L.seg, uniform(xt_a(S.xt)));
    write_resource(p, L.seg, sf.rs, sf.cl, d.v);
  }
  return true;
}

__global__ __launch_bounds__(256) void k_large_flow(DevParams p, FlowState F, int32_t* glist, int32_t* gcount) {
  __shared__ FlLds S;
  const int t = threadIdx.x;
  const uint32_t B = (uint32_t)F.batch;  // tickets taken per counter add (one address: adds serialise)
  uint32_t* tk = F.ticket + (F.epoch & 1);
  if (t == 0) {
    // the other counter was used by the previous launch (stream order: it is done)
    if (blockIdx.x == 0) __hip_atomic_store((gu32*)(F.ticket + ((F.epoch + 1) & 1)), 0u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    S.next = __hip_atomic_fetch_add((gu32*)tk, B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  uint32_t cur = __builtin_amdgcn_readfirstlane(S.next);
  uint32_t end = cur + B;
  while (cur < (uint32_t)F.ntasks) {
    uint32_t nxt = 0;
    const bool first = cur + B == end;
    if (t == 0 && first) nxt = __hip_atomic_fetch_add((gu32*)tk, B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t d = F.tasks[cur];
    const int c = (int)(d & 0x3FFFFFFFu);
    bool ok;
    switch (d >> 30) {
      case kFlowA: ok = fl_task_a(p, F, c, S, glist, gcount); break;
      case kFlowB: ok = fl_task_b(p, F, c, S); break;
      case kFlowC: ok = fl_task_c(p, F, c, S); break;
      default: ok = fl_task_m(p, F, c, S); break;
    }
    if (!ok) return;  // a wait gave up (error word set): stop taking tasks
    __syncthreads();  // every thread is past the task's LDS use
    if (t == 0 && first) S.next = nxt;
    __syncthreads();
    cur += 1;
    if (cur == end || cur >= (uint32_t)F.ntasks) {
      cur = __builtin_amdgcn_readfirstlane(S.next);
      end = cur + B;
    }
  }
}

hipError_t launch_large_flow(const DevParams& p, const FlowState& F, int grid, int32_t* glist, int32_t* gcount,
                             hipStream_t st) {
  if (F.ntasks <= 0 || grid <= 0) return hipSuccess;
  k_large_flow<<<grid, 256, 0, st>>>(p, F, glist, gcount);
  return hipGetLastError();
}

hipError_t large_flow_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_large_flow, 256, 0);
}

}  // namespace dm
