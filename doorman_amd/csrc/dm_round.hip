// dm_round.hip — a round of individual requests decided against the store
// (dm_decide): Resource.Decide (go/server/doorman/resource.go:100-113) for every
// request of a round, each against the store as it was before the round.
//
// Unlike the snapshot tick (dm_kernels.hip), where every stored row is its own
// refresh request, a round's request may differ from the row it will replace
// (new wants or subclients, a client-reported has in learning mode) or come from
// a client the store does not hold.  The reference's algorithms then use the
// request's own values for that client (algorithm.go:115 count, :126 deserved
// share, :148 wantExtra, :157 self skipped, :223-225 new client, :263-269 Map
// substitution) and the stored rows for everyone else.  Here one workgroup takes
// one resource with requests: Clean's sums once, then per request the
// reference's loops as workgroup reductions over the resource's live rows
// (fixed reduction tree: deterministic run to run).
#include <hip/hip_runtime.h>

#include "dm_kernel_util.h"

namespace dm {

__global__ __launch_bounds__(256) void k_decide(DevParams p, const ReqItem* __restrict__ items, ReqArgs q) {
  __shared__ Lds<256> lds;
  const ReqItem it = items[blockIdx.x];
  const int seg = it.seg;
  const int64_t lo = p.seg_off[seg], hi = p.seg_off[seg + 1];
  const Res rs = load_res(p, seg);  // running sums (parity mode)
  // Clean (store.go:169-181): the rows it releases, off the running sums
  AggA a = zeroA();
  for (int64_t j = lo + threadIdx.x; j < hi; j += 256) {
    if (p.now > row_expiry(p, j, p.sub[j], rs.follow_exp)) {
      a.cnt += sub_value(p.sub[j]);
      a.h += p.has[j];
      a.w += p.wants[j];
    }
  }
  a = group_reduce<256>(a, OpA(), lds.a);
  const Clean cl = clean_from(p, rs, a);
  const double C = rs.C;
  for (int64_t k = it.qlo; k < it.qhi; ++k) {
    const int64_t row = q.rows[k];
    const double rh = q.has[k], rw = q.wants[k];
    const long long rsub = q.sub[k];
    const bool self_live = !(p.now > row_expiry(p, row, p.sub[row], rs.follow_exp));  // HasClient after Clean
    const double old_h = self_live ? p.has[row] : 0.0;  // store.Get: zero Lease if absent
    const long long old_s = self_live ? (long long)sub_value(p.sub[row]) : 0;
    double g;
    if (rs.learning) {
      g = rh;  // Learn (algorithm.go:297-302)
    } else if (rs.kind == 0) {
      g = rw;  // NoAlgorithm (:66-72)
    } else if (rs.kind == 1) {
      g = minF(C, rw);  // Static (:78-84)
    } else if (rs.kind == 2) {  // ProportionalShare (:213-293)
      const long long cnt = cl.count + (self_live ? 0 : rsub);  // :217-225
      const double eq = C / (double)cnt;                         // :229
      const double epc = eq * (double)rsub;                      // :233
      const double unused = C - cl.sum_has + old_h;              // :239
      if (cl.sum_wants <= C || rw <= epc) {                      // :245
        g = minF(rw, unused);
      } else {
        AggB b{0.0, 0.0, 0};
        for (int64_t j = lo + threadIdx.x; j < hi; j += 256) {  // store.Map (:259-279)
          if (p.now > row_expiry(p, j, p.sub[j], rs.follow_exp)) continue;
          const bool self = j == row;
          const double wv = self ? rw : p.wants[j];
          const long long sv = self ? rsub : (long long)sub_value(p.sub[j]);
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
      const long long cnt = cl.count - old_s + rsub;  // :115
      const double avail = C - cl.sum_has + old_h;    // :120
      const double eq = C / (double)cnt;              // :123
      const double ds = eq * (double)rsub;            // :126
      if (rw <= ds) {                                 // :131
        g = minF(rw, avail);
      } else {
        AggB b{0.0, 0.0, 0};
        for (int64_t j = lo + threadIdx.x; j < hi; j += 256) {  // round 1 (:156-171), self skipped
          if (j == row || p.now > row_expiry(p, j, p.sub[j], rs.follow_exp)) continue;
          const double wj = p.wants[j];
          const long long sj = sub_value(p.sub[j]);
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
          for (int64_t j = lo + threadIdx.x; j < hi; j += 256) {  // round 2 (:192-202)
            if (j == row || p.now > row_expiry(p, j, p.sub[j], rs.follow_exp)) continue;
            const double wj = p.wants[j];
            const long long sj = sub_value(p.sub[j]);
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
    if (threadIdx.x == 0) {
      q.gets[k] = g;
      q.expiry[k] = rs.exp_out;  // Assign: now + lease length (store.go:161)
    }
  }
}

hipError_t launch_decide(const DevParams& p, const ReqItem* items, int nitems, const ReqArgs& q, hipStream_t st) {
  if (nitems <= 0) return hipSuccess;
  k_decide<<<nitems, 256, 0, st>>>(p, items, q);
  return hipGetLastError();
}

}  // namespace dm
