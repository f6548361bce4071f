// dm_round.hip — a round of individual requests decided against the store
// (dm_decide): Resource.Decide (go/server/doorman/resource.go:100-113) for every
// request of a round, in the caller's order, each seeing the Assigns of the
// requests before it on the same resource.
//
// The reference serialises the Decide calls of one resource on res.mu
// (resource.go:103-104); every algorithm ends with store.Assign (algorithm.go:71,
// 83,132,180,204,247,290,300), which updates the row and the running sums
// (store.go:153-167).  The next request's count, available capacity and loops
// over store.Map therefore see the grants made before it, which is what keeps
// the grants of a round within the capacity (two new FairShare clients that each
// want the whole capacity get C and 0, not C twice).
//
// A round's request may differ from the row it will replace (new wants or
// subclients, a client-reported has in learning mode) or come from a client the
// store does not hold.  The reference's algorithms then use the request's own
// values for that client (algorithm.go:115 count, :126 deserved share, :148
// wantExtra, :157 self skipped, :223-225 new client, :263-269 Map substitution)
// and the stored rows for everyone else.
//
// One workgroup takes one resource with requests.  Clean (store.go:169-181)
// runs once: the resource's rows go to a scratch copy (has, wants, subclients;
// -1 marks a row absent after Clean) and the released rows come off the running
// sums.  Then per request: the reference's loops as workgroup reductions over
// the scratch rows (fixed reduction tree: deterministic run to run), and the
// Assign -- the request's row in the scratch copy takes (gets, wants,
// subclients) and the running sums move by the differences, as store.go:156-158.
// The device store itself is not written (dm_server_tick assigns the round's
// leases with dm_store_upsert afterwards).
#include <hip/hip_runtime.h>

#include "dm_kernel_util.h"

namespace dm {

__global__ __launch_bounds__(256) void k_decide(DevParams p, const ReqItem* __restrict__ items, ReqArgs q) {
  __shared__ Lds<256> lds;
  const ReqItem it = items[blockIdx.x];
  if (it.fast > 0 && q.fast[it.fast - 1].ok) return;  // decided by the fast path (dm_decide_fast.hip)
  const int seg = it.seg;
  const int64_t lo = p.seg_off[seg], hi = p.seg_off[seg + 1];
  const int64_t n = hi - lo;
  double* sh_ = q.sc_has + it.scr;
  double* sw_ = q.sc_wants + it.scr;
  int32_t* ss_ = q.sc_sub + it.scr;
  const Res rs = load_res(p, seg);  // running sums (parity mode)
  // Clean (store.go:169-181): the rows it releases, off the running sums; the
  // scratch copy keeps the rows that stay
  AggA a = zeroA();
  for (int64_t j = threadIdx.x; j < n; j += 256) {
    const int32_t raw = p.sub[lo + j];
    const double hj = p.has[lo + j], wj = p.wants[lo + j];
    const bool gone = p.now > row_expiry(p, lo + j, raw, rs.follow_exp);
    if (gone) {
      a.cnt += sub_value(raw);
      a.h += hj;
      a.w += wj;
    }
    sh_[j] = hj;
    sw_[j] = wj;
    ss_[j] = gone ? -1 : sub_value(raw);
  }
  a = group_reduce<256>(a, OpA(), lds.a);  // its barrier also orders the scratch writes
  const Clean cl = clean_from(p, rs, a);
  long long count = cl.count;
  double sum_has = cl.sum_has, sum_wants = cl.sum_wants;
  const double C = rs.C;
  for (int64_t k = it.qlo; k < it.qhi; ++k) {
    const int64_t self = q.rows[k] - lo;
    const double rh = q.has[k], rw = q.wants[k];
    const long long rsub = q.sub[k];
    const int32_t s_self = ss_[self];
    const bool self_live = s_self >= 0;                    // HasClient
    const double old_h = self_live ? sh_[self] : 0.0;      // store.Get: zero Lease if absent
    const double old_w = self_live ? sw_[self] : 0.0;
    const long long old_s = self_live ? (long long)s_self : 0;
    double g;
    if (rs.learning) {
      g = rh;  // Learn (algorithm.go:297-302)
    } else if (rs.kind == 0) {
      g = rw;  // NoAlgorithm (:66-72)
    } else if (rs.kind == 1) {
      g = minF(C, rw);  // Static (:78-84)
    } else if (rs.kind == 2) {  // ProportionalShare (:213-293)
      const long long cnt = count + (self_live ? 0 : rsub);  // :217-225
      const double eq = C / (double)cnt;                      // :229
      const double epc = eq * (double)rsub;                   // :233
      const double unused = C - sum_has + old_h;              // :239
      if (sum_wants <= C || rw <= epc) {                      // :245
        g = minF(rw, unused);
      } else {
        AggB b{0.0, 0.0, 0};
        for (int64_t j = threadIdx.x; j < n; j += 256) {  // store.Map (:259-279)
          const int32_t sj = ss_[j];
          if (sj < 0) continue;
          const bool me = j == self;
          const double wv = me ? rw : sw_[j];
          const long long sv = me ? rsub : (long long)sj;
          const double esp = eq * (double)sv;  // :273
          if (wv < esp)
            b.x += esp - wv;
          else
            b.y += wv - esp;
        }
        b = group_reduce<256>(b, OpB(), lds.b);
        g = minF(epc + (rw - epc) * (b.x / b.y), unused);  // :283,290
      }
    } else {  // FairShare (:95-206)
      const long long cnt = count - old_s + rsub;  // :115
      const double avail = C - sum_has + old_h;    // :120
      const double eq = C / (double)cnt;           // :123
      const double ds = eq * (double)rsub;         // :126
      if (rw <= ds) {                              // :131
        g = minF(rw, avail);
      } else {
        AggB b{0.0, 0.0, 0};
        for (int64_t j = threadIdx.x; j < n; j += 256) {  // round 1 (:156-171), self skipped
          const int32_t sj = ss_[j];
          if (j == self || sj < 0) continue;
          const double wj = sw_[j];
          const double d = (double)sj * eq;  // :160
          if (wj < d)
            b.x += d - wj;
          else if (wj > d)
            b.i += sj;
        }
        b = group_reduce<256>(b, OpB(), lds.b);
        const double dE = (b.x / (double)(rsub + b.i)) * (double)rsub;  // :148,175
        if (rw < ds + dE) {                                             // :179
          g = minF(rw, avail);
        } else {
          const double T = dE + ds;  // :197
          AggC c{0.0, 0};
          for (int64_t j = threadIdx.x; j < n; j += 256) {  // round 2 (:192-202)
            const int32_t sj = ss_[j];
            if (j == self || sj < 0) continue;
            const double wj = sw_[j];
            if (!(wj > (double)sj * eq)) continue;  // wantExtraClients (:165-169)
            if (wj < T)
              c.ee += T - wj;
            else if (wj > T)
              c.sgt += sj;
          }
          c = group_reduce<256>(c, OpC(), lds.c);
          g = minF(ds + dE + (c.ee / (double)(rsub + c.sgt)) * (double)rsub, avail);  // :189,203-204
        }
      }
    }
    // Assign (store.go:153-167): the running sums and the row the next request sees
    sum_has += g - old_h;
    sum_wants += rw - old_w;
    count += rsub - old_s;
    __syncthreads();  // every thread is done reading this request's rows
    if (threadIdx.x == 0) {
      sh_[self] = g;
      sw_[self] = rw;
      ss_[self] = (int32_t)rsub;
      q.gets[k] = g;
      q.expiry[k] = rs.exp_out;  // now + lease length (store.go:161)
    }
    __syncthreads();  // ... and the next one reads the Assign
  }
}

hipError_t launch_decide(const DevParams& p, const ReqItem* items, int nitems, const ReqArgs& q, hipStream_t st) {
  if (nitems <= 0) return hipSuccess;
  k_decide<<<nitems, 256, 0, st>>>(p, items, q);
  return hipGetLastError();
}

}  // namespace dm
