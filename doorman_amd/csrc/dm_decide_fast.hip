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
  const DD z = dd_add(DD{a.zh, a.zl}, DD{b.zh, b.zl});
  return FdScan{x.hi, x.lo, y.hi, y.lo, z.hi, z.lo, a.i + b.i};
}
__device__ __forceinline__ FdScan fd_zero() { return FdScan{0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0}; }
struct OpFd {
  __device__ FdScan operator()(FdScan a, FdScan b) const { return fd_add(a, b); }
  __device__ static FdScan zero() { return fd_zero(); }
};

// The available capacity a = C - sumHas before each request follows
//   a' = C - (sumHas + g - has) = max(a + has - v, 0)     with g = minF(v, a + has)
// (algorithm.go:120,131,179,204 then store.go:156), a map x -> max(x + c, 0); maps of
// the form x -> max(x + A, B) compose into the same form, so every request's a is an
// exclusive scan of them (x -> max(x, -inf) is the identity; -inf as kFdNone, kept finite
// for the double-double sums).
constexpr double kFdNone = -1e307;
__device__ __forceinline__ bool dd_lt(DD a, DD b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
__device__ __forceinline__ FdLind ld_compose(const FdLind& f, const FdLind& g) {  // f first, then g
  const DD a = dd_add(DD{f.ah, f.al}, DD{g.ah, g.al});
  const DD fb = dd_add(DD{f.bh, f.bl}, DD{g.ah, g.al});
  const DD gb = DD{g.bh, g.bl};
  const DD b = dd_lt(fb, gb) ? gb : fb;
  return FdLind{a.hi, a.lo, b.hi, b.lo};
}
struct OpLd {
  __device__ FdLind operator()(FdLind a, FdLind b) const { return ld_compose(a, b); }
  __device__ static FdLind zero() { return FdLind{0.0, 0.0, kFdNone, 0.0}; }
};

// FairShare round 1's per-row terms (algorithm.go:160-169) at d = s0 * equalShare
__device__ __forceinline__ double fs_t(double w, double d) { return w < d ? d - w : 0.0; }
__device__ __forceinline__ long long fs_c(double w, double d, int s0) { return w > d ? s0 : 0; }
// ProportionalShare's (:273-277) at esp = equalShare * s0
__device__ __forceinline__ double ps_x(double w, double e) { return w < e ? e - w : 0.0; }
__device__ __forceinline__ double ps_y(double w, double e) { return w < e ? 0.0 : w - e; }

// ---- deterministic exclusive scans (256 threads; Hillis-Steele in LDS) ----
template <typename T, typename Op>
__device__ __forceinline__ T block_exclusive(T v, T* lds, T* total) {
  Op op;
  const int t = threadIdx.x;
  lds[t] = v;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const T a = t >= off ? lds[t - off] : Op::zero();
    __syncthreads();
    if (t >= off) lds[t] = op(a, lds[t]);
    __syncthreads();
  }
  *total = lds[255];
  const T ex = t > 0 ? lds[t - 1] : Op::zero();
  __syncthreads();
  return ex;
}

// phase 1: each chunk's total (fixed order: 4 per thread, then the thread totals in order)
template <typename T, typename Op>
__global__ __launch_bounds__(256) void k_fd_scan_part(const T* __restrict__ a, int64_t n, T* part, const FastRes* fr) {
  __shared__ T lds[256];
  if (fr && !fr->ok) return;
  Op op;
  const int64_t base = (int64_t)blockIdx.x * kFdChunk + 4 * threadIdx.x;
  T s = Op::zero();
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (base + i < n) s = op(s, a[base + i]);
  T tot;
  (void)block_exclusive<T, Op>(s, lds, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// phase 2: exclusive scan of the chunk totals, starting at init (one workgroup)
template <typename T, typename Op>
__global__ __launch_bounds__(256) void k_fd_scan_top(T* part, int64_t nparts, const T* init, const FastRes* fr) {
  __shared__ T lds[256];
  if (fr && !fr->ok) return;
  Op op;
  T carry = init ? *init : Op::zero();
  for (int64_t b = 0; b < nparts; b += 256) {
    const int64_t i = b + threadIdx.x;
    const T v = i < nparts ? part[i] : Op::zero();
    T tot;
    const T ex = block_exclusive<T, Op>(v, lds, &tot);
    if (i < nparts) part[i] = op(carry, ex);
    carry = op(carry, tot);
  }
}

// phase 3: every element's exclusive prefix, in place
template <typename T, typename Op>
__global__ __launch_bounds__(256) void k_fd_scan_apply(T* a, int64_t n, const T* part, const FastRes* fr) {
  __shared__ T lds[256];
  if (fr && !fr->ok) return;
  Op op;
  const int64_t base = (int64_t)blockIdx.x * kFdChunk + 4 * threadIdx.x;
  T v[4];
  T s = Op::zero();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = base + i < n ? a[base + i] : Op::zero();
    s = op(s, v[i]);
  }
  T tot;
  T run = op(part[blockIdx.x], block_exclusive<T, Op>(s, lds, &tot));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (base + i < n) a[base + i] = run;
    run = op(run, v[i]);
  }
}

template <typename T, typename Op>
static hipError_t fd_scan(T* a, int64_t n, const T* init, T* part, const FastRes* fr, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t np = (n + kFdChunk - 1) / kFdChunk;
  k_fd_scan_part<T, Op><<<(unsigned)np, 256, 0, st>>>(a, n, part, fr);
  k_fd_scan_top<T, Op><<<1, 256, 0, st>>>(part, np, init, fr);
  k_fd_scan_apply<T, Op><<<(unsigned)np, 256, 0, st>>>(a, n, part, fr);
  return hipGetLastError();
}

// ---- the round ----
// Clean (store.go:169-181) of one chunk of the resource's rows into the round's scratch
// copy (as k_decide), with the chunk's partials: released subclients / has / wants,
// the live rows' subclients range, wants the fast path cannot take.
__global__ __launch_bounds__(256) void k_fd_clean(DevParams p, ReqItem it, FastItem fi, ReqArgs q, FastArgs fa) {
  __shared__ Lds<256> lds;
  const int seg = it.seg;
  const int64_t lo = p.seg_off[seg], n = fi.n;
  const Res rs = load_res(p, seg);
  AggA a = zeroA();
  const int64_t j0 = (int64_t)blockIdx.x * kFdRows;
  const int64_t j1 = j0 + kFdRows < n ? j0 + kFdRows : n;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
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
    q.sc_has[it.scr + j] = hj;
    q.sc_wants[it.scr + j] = wj;
    q.sc_sub[it.scr + j] = gone ? -1 : sv;
  }
  a = group_reduce_t0<256>(a, OpA(), lds.a);
  if (threadIdx.x == 0) fa.pc[fi.c0 + blockIdx.x] = FdClean{a.cnt, a.h, a.w, a.smin, a.smax, a.nan, a.nlive};
}

// The resource's Clean from the chunks' partials (fixed order), the rows' verdict and
// the round's constants.  One workgroup.
__global__ __launch_bounds__(256) void k_fd_check(DevParams p, ReqItem it, FastItem fi, int slot, FastArgs fa) {
  __shared__ Lds<256> lds;
  const Res rs = load_res(p, it.seg);
  AggA a = zeroA();
  for (int c = threadIdx.x; c < fi.nch; c += 256) {
    const FdClean x = fa.pc[fi.c0 + c];
    AggA y = zeroA();
    y.cnt = x.cnt;
    y.h = x.h;
    y.w = x.w;
    y.smin = x.smin;
    y.smax = x.smax;
    y.nan = x.bad;
    y.nlive = x.nlive;
    a = OpA()(a, y);
  }
  a = group_reduce_t0<256>(a, OpA(), lds.a);
  if (threadIdx.x != 0) return;
  const Clean cl = clean_from(p, rs, a);
  const double C = rs.C;
  const int s0 = a.smin;
  const bool ok = !rs.learning && (rs.kind == 2 || rs.kind == 3) && a.nlive > 0 && a.smin == a.smax && s0 >= 1 &&
                  !a.nan && cl.count >= 1 && __builtin_fabs(C) <= kFdMaxAbs;
  FastRes r;
  r.ok = 0;
  r.kind = rs.kind;
  r.s0 = s0;
  r.ok0 = ok ? 1 : 0;
  r.bad = 0;
  r.pad = 0;
  r.C = C;
  r.eq = C / (double)cl.count;  // algorithm.go:123,229
  r.d = (double)s0 * r.eq;      // :160 (eq * s0 at :233,273: the same product)
  r.count = cl.count;
  r.nlive = a.nlive;
  r.sum_has = cl.sum_has;
  r.sum_wants = cl.sum_wants;
  r.init = fd_zero();
  r.exp_out = rs.exp_out;
  fa.fr[slot] = r;
}

// Every request asks from a live row with the resource's count and finite wants.
__global__ __launch_bounds__(256) void k_fd_reqcheck(DevParams p, ReqItem it, FastItem fi, int slot, ReqArgs q,
                                                     FastArgs fa) {
  FastRes* fr = fa.fr + slot;
  if (!fr->ok0) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool bad = false;
  if (j < fi.K) {
    const int64_t k = fi.k0 + j;
    const int64_t row = q.rows[k] - p.seg_off[it.seg];
    bad = q.sub[k] != fr->s0 || q.sc_sub[it.scr + row] < 0 || !(__builtin_fabs(q.wants[k]) <= kFdMaxAbs);
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&fr->bad, 1);
}

// The totals over the live rows before the first request (one chunk's partial), and
// (FairShare) the live rows' wants as sort keys (+inf for absent rows).
__global__ __launch_bounds__(256) void k_fd_totals(ReqItem it, FastItem fi, int slot, ReqArgs q, FastArgs fa) {
  __shared__ FdScan red[4];
  const FastRes& frr = fa.fr[slot];
  if (!frr.ok0 || frr.bad) return;
  const double d = frr.d;
  const int s0 = frr.s0;
  const bool fs = frr.kind == 3;
  const int64_t j0 = (int64_t)blockIdx.x * kFdRows;
  const int64_t j1 = j0 + kFdRows < fi.n ? j0 + kFdRows : fi.n;
  FdScan tot = fd_zero();
  for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
    const bool live = q.sc_sub[it.scr + j] >= 0;
    const double w = q.sc_wants[it.scr + j];
    if (live) {
      if (fs) tot = fd_add(tot, FdScan{fs_t(w, d), 0.0, 0.0, 0.0, 0.0, 0.0, fs_c(w, d, s0)});
      else tot = fd_add(tot, FdScan{ps_x(w, d), 0.0, ps_y(w, d), 0.0, 0.0, 0.0, 0});
    }
    if (fs) fa.keys[fi.m0 + j] = live ? w : __builtin_inf();
  }
  tot = group_reduce_t0<256>(tot, OpFd(), red);
  if (threadIdx.x == 0) fa.pt[fi.c0 + blockIdx.x] = tot;
}

// The verdict, and the totals from the chunks' partials (fixed order).
__global__ __launch_bounds__(256) void k_fd_final(FastItem fi, int slot, FastArgs fa) {
  __shared__ FdScan red[4];
  FastRes* fr = fa.fr + slot;
  const bool ok = fr->ok0 && !fr->bad;
  if (!ok) {
    if (threadIdx.x == 0) fr->ok = 0;
    return;
  }
  FdScan tot = fd_zero();
  for (int c = threadIdx.x; c < fi.nch; c += 256) tot = fd_add(tot, fa.pt[fi.c0 + c]);
  tot = group_reduce_t0<256>(tot, OpFd(), red);
  if (threadIdx.x == 0) {
    tot.zh = fr->sum_wants;  // ProportionalShare's sumWants starts at the cleaned store's
    tot.zl = 0.0;
    fr->init = tot;
    fr->ok = 1;
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
    e = FdScan{x.hi, x.lo, 0.0, 0.0, 0.0, 0.0, fs_c(rw, d, fr.s0) - fs_c(pw, d, fr.s0)};
    fa.ev_in[fi.e0 + 2 * j] = rw;
    fa.evs_in[fi.e0 + 2 * j] = 1;
    fa.ev_in[fi.e0 + 2 * j + 1] = pw;
    fa.evs_in[fi.e0 + 2 * j + 1] = -1;
  } else {
    const DD x = dd_two_sum(ps_x(rw, d), -ps_x(pw, d));
    const DD y = dd_two_sum(ps_y(rw, d), -ps_y(pw, d));
    const DD z = dd_two_sum(rw, -pw);  // sumWants moves by the request's wants (store.go:157)
    e = FdScan{x.hi, x.lo, y.hi, y.lo, z.hi, z.lo, 0};
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
  fa.ps[fi.m0 + j] = FdScan{v, 0.0, 0.0, 0.0, 0.0, 0.0, 0};
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
        v[i] = FdScan{x.hi, x.lo, 0.0, 0.0, 0.0, 0.0, es[base + i]};
      }
      s = fd_add(s, v[i]);
    }
    FdScan tot;
    FdScan run = fd_add(carry, block_exclusive<FdScan, OpFd>(s, lds, &tot));
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
// (:179), else round 2 at T (:189-204); ProportionalShare: rw when the store's
// sumWants (the earlier Assigns' included) is within C or rw within its equal share
// (:245), else its round-1 grant (:283).
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
    const double sw = dd_val(DD{e.zh, e.zl});     // sumWants before request k
    v = (sw <= fr.C || rw <= epc) ? rw : epc + (rw - epc) * (x / y);  // :245, :283
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

// Rounds in which some client asks twice: the grant of its earlier request is the has
// its later one sees, so the available capacity (algorithm.go:120,239) after the
// earlier grants (store.go:156) runs in order, on one wave per fast item.  Lanes hold
// 64 requests' inputs; the recurrence walks them with readlanes.
__global__ __launch_bounds__(64) void k_fd_seq(DevParams p, ReqItem it, FastItem fi, int slot, ReqArgs q,
                                               FastArgs fa) {
  __shared__ double gl[64];
  const FastRes& frr = fa.fr[slot];
  if (!frr.ok) return;
  const FastRes fr = frr;
  const int lane = threadIdx.x;
  const int64_t lo = p.seg_off[it.seg];
  const double C = fr.C;
  double sh = fr.sum_has;
  const int64_t end = fi.k0 + fi.K;
  for (int64_t base = fi.k0; base < end; base += 64) {
    const int64_t k = base + lane;
    const bool in = k < end;
    const int64_t kc = in ? k : base;
    const double v = fa.v[kc];
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
      const double g = minF(vi, avail);
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

// Rounds in which every client asks once: the available capacity before each request
// from the exclusive composition of the maps x -> max(x + has - v, 0) (OpLd).
__global__ __launch_bounds__(256) void k_fd_lind_fill(DevParams p, ReqItem it, FastItem fi, int slot, ReqArgs q,
                                                      FastArgs fa) {
  if (!fa.fr[slot].ok) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= fi.K) return;
  const int64_t k = fi.k0 + j;
  const double oh = q.sc_has[it.scr + (q.rows[k] - p.seg_off[it.seg])];  // store.Get(self).Has
  const DD c = dd_two_sum(oh, -fa.v[k]);
  fa.ld[k] = FdLind{c.hi, c.lo, 0.0, 0.0};
}

__global__ __launch_bounds__(256) void k_fd_lind_final(DevParams p, ReqItem it, FastItem fi, int slot, ReqArgs q,
                                                       FastArgs fa) {
  const FastRes& fr = fa.fr[slot];
  if (!fr.ok) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= fi.K) return;
  const int64_t k = fi.k0 + j;
  const double oh = q.sc_has[it.scr + (q.rows[k] - p.seg_off[it.seg])];
  const FdLind f = fa.ld[k];
  const DD a0 = dd_two_sum(fr.C, -fr.sum_has);  // C - sumHas before the round
  const DD x = dd_add(a0, DD{f.ah, f.al});
  const DD b = DD{f.bh, f.bl};
  const DD a = dd_lt(x, b) ? b : x;                  // C - sumHas before request k
  const double avail = dd_val(dd_add(a, dd_of(oh)));  // algorithm.go:120,239
  q.gets[k] = minF(fa.v[k], avail);                   // :131,179,204,245,290
  q.expiry[k] = fr.exp_out;                           // now + lease length (store.go:161)
}

// ---- host side ----
// Clean, the verdict and the round's totals of one fast item.
hipError_t fd_rows(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                   const FastArgs& fa, hipStream_t st) {
  const unsigned gk = (unsigned)((fi.K + 255) / 256);
  k_fd_clean<<<(unsigned)fi.nch, 256, 0, st>>>(p, it, fi, q, fa);
  k_fd_check<<<1, 256, 0, st>>>(p, it, fi, slot, fa);
  k_fd_reqcheck<<<gk, 256, 0, st>>>(p, it, fi, slot, q, fa);
  k_fd_totals<<<(unsigned)fi.nch, 256, 0, st>>>(it, fi, slot, q, fa);
  k_fd_final<<<1, 256, 0, st>>>(fi, slot, fa);
  return hipGetLastError();
}

// Each request's Assign delta and the running totals before it (a scan).
hipError_t fd_item(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                   const FastArgs& fa, FdScan* part, hipStream_t st) {
  const unsigned gk = (unsigned)((fi.K + 255) / 256);
  k_fd_delta<<<gk, 256, 0, st>>>(p, it, fi, slot, q, fa);
  return fd_scan<FdScan, OpFd>(fa.sc + fi.k0, fi.K, &fa.fr[slot].init, part, fa.fr + slot, st);
}

// After the sorts: FairShare's round-2 structures (the kernels return at once for
// ProportionalShare), every request's grant before the cap, then the cap itself.
hipError_t fd_item_sorted(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                          const FastArgs& fa, FdScan* part, hipStream_t st) {
  const unsigned gk = (unsigned)((fi.K + 255) / 256);
  k_fd_m0_fill<<<(unsigned)((fi.n + 1 + 255) / 256), 256, 0, st>>>(fi, slot, fa);
  hipError_t e = fd_scan<FdScan, OpFd>(fa.ps + fi.m0, fi.n + 1, nullptr, part, fa.fr + slot, st);
  if (e != hipSuccess) return e;
  k_fd_ev_prefix<<<(unsigned)fi.nblk, 256, 0, st>>>(fi, slot, fa);
  k_fd_query<<<gk, 256, 0, st>>>(it, fi, slot, q, fa);
  if (fi.repeats) {
    k_fd_seq<<<1, 64, 0, st>>>(p, it, fi, slot, q, fa);
    return hipGetLastError();
  }
  k_fd_lind_fill<<<gk, 256, 0, st>>>(p, it, fi, slot, q, fa);
  e = fd_scan<FdLind, OpLd>(fa.ld + fi.k0, fi.K, nullptr, reinterpret_cast<FdLind*>(part), fa.fr + slot, st);
  if (e != hipSuccess) return e;
  k_fd_lind_final<<<gk, 256, 0, st>>>(p, it, fi, slot, q, fa);
  return hipGetLastError();
}

// The items' initial wants (one radix sort each: a segmented sort gives a segment one
// workgroup), and every event block (segmented: 4096 events each).  hipCUB radix
// sorts are stable and deterministic.  temp == nullptr: *bytes = the storage needed.
hipError_t fd_sort_keys(void* temp, size_t* bytes, const double* in, double* out, int64_t n, hipStream_t st) {
  return hipcub::DeviceRadixSort::SortKeys(temp, *bytes, in, out, (int)n, 0, (int)(8 * sizeof(double)), st);
}
hipError_t fd_sort_pairs(void* temp, size_t* bytes, const double* kin, double* kout, const int32_t* vin,
                         int32_t* vout, int64_t n, int nseg, const int64_t* begin, const int64_t* end,
                         hipStream_t st) {
  return hipcub::DeviceSegmentedRadixSort::SortPairs(temp, *bytes, kin, kout, vin, vout, (int)n, nseg, begin, end, 0,
                                                     (int)(8 * sizeof(double)), st);
}

}  // namespace dm
