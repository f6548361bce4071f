// dm_decide_fast.hip — dm_decide for a resource with many requests in one round.
//
// k_decide (dm_round.hip) replays Resource.Decide request by request
// (go/server/doorman/resource.go:100-113): every FairShare / ProportionalShare
// request above its deserved share walks the whole store (store.Map,
// algorithm.go:156-171,192-202,259-279) and then assigns (store.go:153-167), so a
// round of K requests on an n-client resource costs O(K n) on one workgroup.
//
// When every request keeps the counts -- each requester is a live row of the store
// (after Clean) asking with the subclients count that every live row holds -- the
// count, and with it equalShare = C / count (:123, :229), is the same for the whole
// round.  Then, per request k (self = its row, w_k = the row's wants before it):
//   FairShare round 1 (:156-171, self skipped):
//       extra_k      = X_k - t(w_k),   X_k = sum over live rows of t(w) = [w < d](d - w)
//       wantExtra_k  = I_k - c(w_k),   I_k = sum over live rows of c(w) = [w > d] s0
//     and every Assign moves X / I by its own row only: X_{k+1} = X_k + t(rw_k) - t(w_k),
//     so X_k, I_k are exclusive prefix sums over the round's requests (a scan);
//   FairShare round 2 at T_k (:192-202):
//       extraExtra_k = sum over d < w < T_k of (T_k - w)  = cnt * T_k - sum(w)
//       (the algebraic form) and wantExtraExtra_k = s0 * #{w > T_k},
//     counted over the wants as the earlier Assigns left them (self excluded):
//     the sorted initial wants plus the round's Assign events (the request's wants in,
//     the row's previous wants out) before k, sorted per block of kFdBlock requests;
//   ProportionalShare (:259-279, self with its request values): the same prefix sums.
// Only the available capacity C - sumHas + has (:120, :239) depends on the earlier
// grants (and ProportionalShare's sumWants <= C test, :245, on the earlier wants):
// one wave runs that recurrence over the round in order.  O((n + K) log) work
// instead of O(K n).  Sums are double-double (the scans) or the algebraic form, so
// results agree with the literal replay within the survey's tolerance, not bit for
// bit; the order of every sum is fixed, so they are deterministic.
//
// Any other round (counts change, a new client, learning mode, NaN / huge wants) is
// left to k_decide (FastRes::ok = 0).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "dm_kernel_util.h"

namespace dm {

// ---- double-double sums (Knuth's TwoSum; the build has -ffp-contract=off) ----
struct DD {
  double hi, lo;
};
__device__ __forceinline__ DD dd_two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return DD{s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ DD dd_add(DD a, DD b) {
  const DD s = dd_two_sum(a.hi, b.hi);
  const double e = s.lo + (a.lo + b.lo);
  const double hi = s.hi + e;
  return DD{hi, e - (hi - s.hi)};
}
__device__ __forceinline__ DD dd_of(double v) { return DD{v, 0.0}; }
__device__ __forceinline__ double dd_val(DD a) { return a.hi + a.lo; }

__device__ __forceinline__ FdScan fd_add(const FdScan& a, const FdScan& b) {
  const DD x = dd_add(DD{a.xh, a.xl}, DD{b.xh, b.xl});
  const DD y = dd_add(DD{a.yh, a.yl}, DD{b.yh, b.yl});
  return FdScan{x.hi, x.lo, y.hi, y.lo, a.i + b.i};
}
struct OpFd {
  __device__ FdScan operator()(FdScan a, FdScan b) const { return fd_add(a, b); }
};
__device__ __forceinline__ FdScan fd_zero() { return FdScan{0.0, 0.0, 0.0, 0.0, 0}; }

// FairShare round 1's per-row terms (algorithm.go:160-169) at d = s0 * equalShare
__device__ __forceinline__ double fs_t(double w, double d) { return w < d ? d - w : 0.0; }
__device__ __forceinline__ long long fs_c(double w, double d, int s0) { return w > d ? s0 : 0; }
// ProportionalShare's (:273-277) at esp = equalShare * s0
__device__ __forceinline__ double ps_x(double w, double e) { return w < e ? e - w : 0.0; }
__device__ __forceinline__ double ps_y(double w, double e) { return w < e ? 0.0 : w - e; }

// ---- block-wide exclusive scan of FdScan (256 threads; Hillis-Steele in LDS) ----
__device__ __forceinline__ FdScan block_exclusive(FdScan v, FdScan* lds, FdScan* total) {
  const int t = threadIdx.x;
  lds[t] = v;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const FdScan a = t >= off ? lds[t - off] : fd_zero();
    __syncthreads();
    if (t >= off) lds[t] = fd_add(a, lds[t]);
    __syncthreads();
  }
  *total = lds[255];
  const FdScan ex = t > 0 ? lds[t - 1] : fd_zero();
  __syncthreads();
  return ex;
}


// phase 1: each chunk's total (fixed order: 4 per thread, then the thread totals in order)
__global__ __launch_bounds__(256) void k_fd_scan_part(const FdScan* __restrict__ a, int64_t n, FdScan* part,
                                                      const FastRes* fr) {
  __shared__ FdScan lds[256];
  if (fr && !fr->ok) return;
  const int64_t base = (int64_t)blockIdx.x * kFdChunk + 4 * threadIdx.x;
  FdScan s = fd_zero();
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (base + i < n) s = fd_add(s, a[base + i]);
  FdScan tot;
  (void)block_exclusive(s, lds, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// phase 2: exclusive scan of the chunk totals, starting at init (one workgroup)
__global__ __launch_bounds__(256) void k_fd_scan_top(FdScan* part, int64_t nparts, const FdScan* init,
                                                     const FastRes* fr) {
  __shared__ FdScan lds[256];
  if (fr && !fr->ok) return;
  FdScan carry = init ? *init : fd_zero();
  for (int64_t b = 0; b < nparts; b += 256) {
    const int64_t i = b + threadIdx.x;
    const FdScan v = i < nparts ? part[i] : fd_zero();
    FdScan tot;
    const FdScan ex = block_exclusive(v, lds, &tot);
    if (i < nparts) part[i] = fd_add(carry, ex);
    carry = fd_add(carry, tot);
  }
}

// phase 3: every element's exclusive prefix, in place
__global__ __launch_bounds__(256) void k_fd_scan_apply(FdScan* a, int64_t n, const FdScan* part, const FastRes* fr) {
  __shared__ FdScan lds[256];
  if (fr && !fr->ok) return;
  const int64_t base = (int64_t)blockIdx.x * kFdChunk + 4 * threadIdx.x;
  FdScan v[4];
  FdScan s = fd_zero();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = base + i < n ? a[base + i] : fd_zero();
    s = fd_add(s, v[i]);
  }
  FdScan tot;
  FdScan run = fd_add(part[blockIdx.x], block_exclusive(s, lds, &tot));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (base + i < n) a[base + i] = run;
    run = fd_add(run, v[i]);
  }
}

static hipError_t fd_scan(FdScan* a, int64_t n, const FdScan* init, FdScan* part, const FastRes* fr,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t np = (n + kFdChunk - 1) / kFdChunk;
  k_fd_scan_part<<<(unsigned)np, 256, 0, st>>>(a, n, part, fr);
  k_fd_scan_top<<<1, 256, 0, st>>>(part, np, init, fr);
  k_fd_scan_apply<<<(unsigned)np, 256, 0, st>>>(a, n, part, fr);
  return hipGetLastError();
}

// ---- the round ----
// Clean into the round's scratch copy (as k_decide), the eligibility test, and the
// totals over the live rows before the first request.  One workgroup per fast item.
__global__ __launch_bounds__(256) void k_fd_prep(DevParams p, const ReqItem* __restrict__ items, ReqArgs q,
                                                 FastArgs fa) {
  __shared__ Lds<256> lds;
  __shared__ FdScan red[4];
  const FastItem fi = fa.fi[blockIdx.x];
  const ReqItem it = items[fi.item];
  const int seg = it.seg;
  const int64_t lo = p.seg_off[seg], n = p.seg_off[seg + 1] - lo;
  double* sh_ = q.sc_has + it.scr;
  double* sw_ = q.sc_wants + it.scr;
  int32_t* ss_ = q.sc_sub + it.scr;
  const Res rs = load_res(p, seg);
  AggA a = zeroA();
  for (int64_t j = threadIdx.x; j < n; j += 256) {
    const int32_t raw = p.sub[lo + j];
    const double hj = p.has[lo + j], wj = p.wants[lo + j];
    const bool gone = p.now > row_expiry(p, lo + j, raw, rs.follow_exp);
    const int sv = sub_value(raw);
    if (gone) {
      a.cnt += sv;
      a.h += hj;
      a.w += wj;
    } else {
      a.smin = sv < a.smin ? sv : a.smin;
      a.smax = sv > a.smax ? sv : a.smax;
      a.nan |= !(__builtin_fabs(wj) <= kFdMaxAbs) ? 1 : 0;  // NaN, infinite or huge wants
      a.nlive += 1;
    }
    sh_[j] = hj;
    sw_[j] = wj;
    ss_[j] = gone ? -1 : sv;
  }
  a = group_reduce<256>(a, OpA(), lds.a);  // its barriers also order the scratch writes
  const Clean cl = clean_from(p, rs, a);
  const double C = rs.C;
  const int s0 = a.smin;
  bool ok = !rs.learning && (rs.kind == 2 || rs.kind == 3) && a.nlive > 0 && a.smin == a.smax && s0 >= 1 &&
            !a.nan && cl.count >= 1 && __builtin_fabs(C) <= kFdMaxAbs;
  int bad = ok ? 0 : 1;
  for (int64_t k = it.qlo + threadIdx.x; ok && k < it.qhi; k += 256) {
    const int64_t row = q.rows[k] - lo;
    if (q.sub[k] != s0 || ss_[row] < 0 || !(__builtin_fabs(q.wants[k]) <= kFdMaxAbs)) bad = 1;
  }
  ok = !__syncthreads_or(bad);
  const double eq = C / (double)cl.count;  // algorithm.go:123,229
  const double d = (double)s0 * eq;        // :160 (eq * s0 at :233,273: the same product)
  FdScan tot = fd_zero();
  if (ok) {
    for (int64_t j = threadIdx.x; j < n; j += 256) {
      const bool live = ss_[j] >= 0;
      const double w = sw_[j];
      if (live) {
        if (rs.kind == 3) {
          tot = fd_add(tot, FdScan{fs_t(w, d), 0.0, 0.0, 0.0, fs_c(w, d, s0)});
        } else {
          tot = fd_add(tot, FdScan{ps_x(w, d), 0.0, ps_y(w, d), 0.0, 0});
        }
      }
      if (rs.kind == 3) fa.keys[fi.m0 + j] = live ? w : __builtin_inf();
    }
    tot = group_reduce<256>(tot, OpFd(), red);
  }
  if (threadIdx.x == 0) {
    FastRes r;
    r.ok = ok ? 1 : 0;
    r.kind = rs.kind;
    r.s0 = s0;
    r.pad = 0;
    r.C = C;
    r.eq = eq;
    r.d = d;
    r.count = cl.count;
    r.nlive = a.nlive;
    r.sum_has = cl.sum_has;
    r.sum_wants = cl.sum_wants;
    r.init = tot;
    r.exp_out = rs.exp_out;
    fa.fr[blockIdx.x] = r;
  }
}

// Per request: the row's wants before it, the delta its Assign makes to the running
// totals, and (FairShare) its two Assign events.
__global__ __launch_bounds__(256) void k_fd_delta(DevParams p, ReqItem it, FastItem fi, int slot, ReqArgs q,
                                                  FastArgs fa) {
  const FastRes& fr = fa.fr[slot];
  if (!fr.ok) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= fi.K) return;
  const int64_t k = fi.k0 + j;
  const int64_t lo = p.seg_off[it.seg];
  const int64_t prev = fa.prev[k];
  const double rw = q.wants[k];
  const double pw = prev >= 0 ? q.wants[prev] : q.sc_wants[it.scr + (q.rows[k] - lo)];
  fa.pw[k] = pw;
  const double d = fr.d;
  FdScan e;
  if (fr.kind == 3) {
    const DD x = dd_two_sum(fs_t(rw, d), -fs_t(pw, d));
    e = FdScan{x.hi, x.lo, 0.0, 0.0, fs_c(rw, d, fr.s0) - fs_c(pw, d, fr.s0)};
    fa.ev_in[fi.e0 + 2 * j] = rw;
    fa.evs_in[fi.e0 + 2 * j] = 1;
    fa.ev_in[fi.e0 + 2 * j + 1] = pw;
    fa.evs_in[fi.e0 + 2 * j + 1] = -1;
  } else {
    const DD x = dd_two_sum(ps_x(rw, d), -ps_x(pw, d));
    const DD y = dd_two_sum(ps_y(rw, d), -ps_y(pw, d));
    e = FdScan{x.hi, x.lo, y.hi, y.lo, 0};
  }
  fa.sc[k] = e;
}

// The sorted wants as scan input: value j for j < nlive, 0 after (the exclusive scan
// over n + 1 entries then holds every prefix sum, the total at nlive and beyond).
__global__ __launch_bounds__(256) void k_fd_m0_fill(FastItem fi, int slot, FastArgs fa) {
  const FastRes& fr = fa.fr[slot];
  if (!fr.ok || fr.kind != 3) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j > fi.n) return;
  const double v = j < fr.nlive ? fa.keys_s[fi.m0 + j] : 0.0;
  fa.ps[fi.m0 + j] = FdScan{v, 0.0, 0.0, 0.0, 0};
}

// Per event block: exclusive prefix counts / sums of its sorted events, and its
// events <= d.  One workgroup per block.
__global__ __launch_bounds__(256) void k_fd_ev_prefix(FastItem fi, int slot, FastArgs fa) {
  __shared__ FdScan lds[256];
  const FastRes& fr = fa.fr[slot];
  if (!fr.ok || fr.kind != 3) return;
  const int64_t b = blockIdx.x;
  const int64_t len = 2 * std::min<int64_t>(kFdBlock, fi.K - b * kFdBlock);
  const double* ev = fa.ev + fi.e0 + 2 * b * kFdBlock;
  const int32_t* es = fa.evs + fi.e0 + 2 * b * kFdBlock;
  const int64_t po = (fi.b0 + b) * (2 * kFdBlock + 1);
  FdScan carry = fd_zero();
  for (int64_t c = 0; c < len; c += kFdChunk) {
    const int64_t base = c + 4 * threadIdx.x;
    FdScan v[4], s = fd_zero();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = fd_zero();
      if (base + i < len) {
        const DD x = dd_of(es[base + i] > 0 ? ev[base + i] : -ev[base + i]);
        v[i] = FdScan{x.hi, x.lo, 0.0, 0.0, es[base + i]};
      }
      s = fd_add(s, v[i]);
    }
    FdScan tot;
    FdScan run = fd_add(carry, block_exclusive(s, lds, &tot));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (base + i <= len) {
        fa.ecnt[po + base + i] = (int32_t)run.i;
        fa.esum[po + base + i] = double2{run.xh, run.xl};
      }
      run = fd_add(run, v[i]);
    }
    carry = fd_add(carry, tot);
  }
  __syncthreads();  // every prefix written before thread 0 reads them
  if (threadIdx.x == 0) {
    if (len % kFdChunk == 0) {  // the total at index len (no thread's slot reached it)
      fa.ecnt[po + len] = (int32_t)carry.i;
      fa.esum[po + len] = double2{carry.xh, carry.xl};
    }
    int64_t a = 0, z = len;  // upper_bound(d)
    while (a < z) {
      const int64_t m = (a + z) >> 1;
      if (ev[m] <= fr.d) a = m + 1;
      else z = m;
    }
    fa.bdc[fi.b0 + b] = fa.ecnt[po + a];
    fa.bds[fi.b0 + b] = fa.esum[po + a];
  }
}

__device__ __forceinline__ int64_t lower_bound_d(const double* a, int64_t n, double v) {  // first a[i] >= v
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1;
    else hi = m;
  }
  return lo;
}
__device__ __forceinline__ int64_t upper_bound_d(const double* a, int64_t n, double v) {  // first a[i] > v
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] <= v) lo = m + 1;
    else hi = m;
  }
  return lo;
}

// Per request: its grant before the available-capacity cap.  FairShare: rw when it
// is within deservedShare (algorithm.go:131) or deservedShare + deservedExtra
// (:179), else round 2 at T (:189-204); ProportionalShare: its round-1 grant
// (:283), used only when sumWants > C (the recurrence decides).
__global__ __launch_bounds__(256) void k_fd_query(ReqItem it, FastItem fi, int slot, ReqArgs q, FastArgs fa) {
  const FastRes& frr = fa.fr[slot];
  if (!frr.ok) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= fi.K) return;
  const FastRes fr = frr;
  const int64_t k = fi.k0 + j;
  const double rw = q.wants[k], pw = fa.pw[k];
  const FdScan e = fa.sc[k];  // the running totals before request k
  const int s0 = fr.s0;
  const double rsub = (double)s0;
  const double eq = fr.eq, d = fr.d;
  double v;
  if (fr.kind == 2) {  // ProportionalShare: the store's rows with request k's values for its row
    const double x = dd_val(dd_add(dd_add(DD{e.xh, e.xl}, dd_of(-ps_x(pw, d))), dd_of(ps_x(rw, d))));
    const double y = dd_val(dd_add(dd_add(DD{e.yh, e.yl}, dd_of(-ps_y(pw, d))), dd_of(ps_y(rw, d))));
    const double epc = eq * rsub;                 // :233
    v = epc + (rw - epc) * (x / y);               // :283
  } else {
    const double ds = eq * rsub;  // :126
    if (rw <= ds) {
      v = rw;  // :131
    } else {
      const double x = dd_val(dd_add(DD{e.xh, e.xl}, dd_of(-fs_t(pw, d))));  // self skipped (:157)
      const long long wi = e.i - fs_c(pw, d, s0);
      const double dE = (x / (double)(s0 + wi)) * rsub;  // :148,175
      if (rw < ds + dE) {
        v = rw;  // :179
      } else {
        const double T = dE + ds;  // :197
        // the wants as the Assigns before k left them: sorted initial wants ...
        const double* M = fa.keys_s + fi.m0;
        const int64_t nl = fr.nlive;
        const int64_t lt = lower_bound_d(M, nl, T), le = upper_bound_d(M, nl, T), ld = upper_bound_d(M, nl, d);
        long long c_lt = lt, c_le = le, c_ld = ld;
        DD s_lt = DD{fa.ps[fi.m0 + lt].xh, fa.ps[fi.m0 + lt].xl};
        DD s_ld = DD{fa.ps[fi.m0 + ld].xh, fa.ps[fi.m0 + ld].xl};
        // ... plus every earlier block's events ...
        const int64_t bk = j / kFdBlock;
        for (int64_t bb = 0; bb < bk; ++bb) {
          const double* ev = fa.ev + fi.e0 + 2 * bb * kFdBlock;
          const int64_t po = (fi.b0 + bb) * (2 * kFdBlock + 1);
          const int64_t l = lower_bound_d(ev, 2 * kFdBlock, T), u = upper_bound_d(ev, 2 * kFdBlock, T);
          c_lt += fa.ecnt[po + l];
          const double2 sl = fa.esum[po + l];
          s_lt = dd_add(s_lt, DD{sl.x, sl.y});
          c_le += fa.ecnt[po + u];
          c_ld += fa.bdc[fi.b0 + bb];
          const double2 sd = fa.bds[fi.b0 + bb];
          s_ld = dd_add(s_ld, DD{sd.x, sd.y});
        }
        // ... plus this block's requests before k
        for (int64_t kk = fi.k0 + bk * kFdBlock; kk < k; ++kk) {
          const double a = q.wants[kk], r = fa.pw[kk];
          if (a < T) {
            c_lt += 1;
            s_lt = dd_add(s_lt, dd_of(a));
          }
          if (a <= T) c_le += 1;
          if (a <= d) {
            c_ld += 1;
            s_ld = dd_add(s_ld, dd_of(a));
          }
          if (r < T) {
            c_lt -= 1;
            s_lt = dd_add(s_lt, dd_of(-r));
          }
          if (r <= T) c_le -= 1;
          if (r <= d) {
            c_ld -= 1;
            s_ld = dd_add(s_ld, dd_of(-r));
          }
        }
        long long cin = T > d ? c_lt - c_ld : 0;
        DD sin = T > d ? dd_add(s_lt, DD{-s_ld.hi, -s_ld.lo}) : dd_of(0.0);
        long long gt = fr.nlive - c_le;
        if (d < pw && pw < T) {  // self (:157 round-2 loop skips it too)
          cin -= 1;
          sin = dd_add(sin, dd_of(-pw));
        }
        if (pw > T) gt -= 1;
        const double ee = (double)cin * T - dd_val(sin);  // extraExtra (:197-198), algebraic
        const long long sgt = (long long)s0 * gt;         // (:199-200)
        v = ds + dE + (ee / (double)(s0 + sgt)) * rsub;   // :189,203-204
      }
    }
  }
  fa.v[k] = v;
}

// The round in order (one wave per fast item): the available capacity after the
// earlier grants (algorithm.go:120,239), ProportionalShare's sumWants test (:245),
// the Assigns' running sums (store.go:156-158).  Lanes hold 64 requests' inputs;
// the recurrence walks them with readlanes.
__global__ __launch_bounds__(64) void k_fd_seq(DevParams p, ReqItem it, FastItem fi, int slot, ReqArgs q,
                                               FastArgs fa) {
  __shared__ double gl[64];
  const FastRes& frr = fa.fr[slot];
  if (!frr.ok) return;
  const FastRes fr = frr;
  const int lane = threadIdx.x;
  const int64_t lo = p.seg_off[it.seg];
  const double C = fr.C;
  const bool ps = fr.kind == 2;
  const double epc = fr.eq * (double)fr.s0;
  double sh = fr.sum_has, sw = fr.sum_wants;
  const int64_t end = fi.k0 + fi.K;
  for (int64_t base = fi.k0; base < end; base += 64) {
    const int64_t k = base + lane;
    const bool in = k < end;
    const int64_t kc = in ? k : base;
    const double v = fa.v[kc], rw = q.wants[kc], pw = fa.pw[kc];
    const int64_t prev = fa.prev[kc];
    const double oh0 = prev < 0 ? q.sc_has[it.scr + (q.rows[kc] - lo)] : 0.0;
    const int m = (int)std::min<int64_t>(64, end - base);
    for (int i = 0; i < m; ++i) {
      const int64_t pv = readlane_any(prev, i);
      double oh;  // store.Get(self).Has: the stored has, or the grant of this row's earlier request
      if (pv < 0) oh = readlane_any(oh0, i);
      else if (pv >= base) oh = gl[pv - base];
      else oh = ld_wt(q.gets + pv);
      const double vi = readlane_any(v, i);
      const double avail = C - sh + oh;
      double g;
      if (ps) {
        const double rwi = readlane_any(rw, i);
        g = (sw <= C || rwi <= epc) ? minF(rwi, avail) : minF(vi, avail);
        sw += rwi - readlane_any(pw, i);
      } else {
        g = minF(vi, avail);
        // (sumWants moves too, store.go:157, but nothing in FairShare reads it)
      }
      sh += g - oh;
      if (lane == 0) gl[i] = g;
    }
    __syncthreads();
    if (in) {
      st_wt(q.gets + k, gl[lane]);
      q.expiry[k] = fr.exp_out;  // now + lease length (store.go:161)
    }
    __syncthreads();
  }
}

// ---- host side ----
hipError_t fd_prep(const DevParams& p, const ReqItem* items, const ReqArgs& q, const FastArgs& fa, int nfast,
                   hipStream_t st) {
  if (nfast <= 0) return hipSuccess;
  k_fd_prep<<<nfast, 256, 0, st>>>(p, items, q, fa);
  return hipGetLastError();
}

hipError_t fd_item(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                   const FastArgs& fa, FdScan* part, hipStream_t st) {
  const unsigned gk = (unsigned)((fi.K + 255) / 256);
  k_fd_delta<<<gk, 256, 0, st>>>(p, it, fi, slot, q, fa);
  hipError_t e = fd_scan(fa.sc + fi.k0, fi.K, &fa.fr[slot].init, part, fa.fr + slot, st);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t fd_item_sorted(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                          const FastArgs& fa, FdScan* part, hipStream_t st) {
  const unsigned gk = (unsigned)((fi.K + 255) / 256);
  // FairShare's round-2 structures (the kernels return at once for ProportionalShare)
  k_fd_m0_fill<<<(unsigned)((fi.n + 1 + 255) / 256), 256, 0, st>>>(fi, slot, fa);
  hipError_t e = fd_scan(fa.ps + fi.m0, fi.n + 1, nullptr, part, fa.fr + slot, st);
  if (e != hipSuccess) return e;
  k_fd_ev_prefix<<<(unsigned)fi.nblk, 256, 0, st>>>(fi, slot, fa);
  k_fd_query<<<gk, 256, 0, st>>>(it, fi, slot, q, fa);
  k_fd_seq<<<1, 64, 0, st>>>(p, it, fi, slot, q, fa);
  return hipGetLastError();
}

// Segmented sorts (hipCUB radix sorts: stable, deterministic): the items' initial
// wants, and every event block.  temp == nullptr: *bytes = the storage needed.
hipError_t fd_sort_keys(void* temp, size_t* bytes, const double* in, double* out, int64_t n, int nseg,
                        const int64_t* begin, const int64_t* end, hipStream_t st) {
  return hipcub::DeviceSegmentedRadixSort::SortKeys(temp, *bytes, in, out, (int)n, nseg, begin, end, 0,
                                                    (int)(8 * sizeof(double)), st);
}
hipError_t fd_sort_pairs(void* temp, size_t* bytes, const double* kin, double* kout, const int32_t* vin,
                         int32_t* vout, int64_t n, int nseg, const int64_t* begin, const int64_t* end,
                         hipStream_t st) {
  return hipcub::DeviceSegmentedRadixSort::SortPairs(temp, *bytes, kin, kout, vin, vout, (int)n, nseg, begin, end, 0,
                                                     (int)(8 * sizeof(double)), st);
}

}  // namespace dm
