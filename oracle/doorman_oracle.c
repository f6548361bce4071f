/*
 * doorman_oracle.c — CPU restatement of Doorman's lease algorithms.
 * TEST INFRASTRUCTURE ONLY (see doorman_oracle.h).  Never linked into the product.
 *
 * Every function cites the reference statement it restates
 * (paths relative to the reference repository root).
 */
#include "doorman_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* store.go:105-111 leaseStoreImpl.  The Go map[string]Lease becomes a dense   */
/* array indexed by client id with a presence flag; Map/Clean iterate in      */
/* ascending id order (Go's order is random, so this is one valid execution). */
/* ------------------------------------------------------------------------- */
struct or_store {
  int64_t cap;
  or_lease* leases;
  unsigned char* present;
  double sum_wants;
  double sum_has;
  int64_t count;
};

or_store* or_store_new(int64_t max_clients) {
  or_store* s = (or_store*)calloc(1, sizeof(or_store));
  s->cap = max_clients > 0 ? max_clients : 1;
  s->leases = (or_lease*)calloc((size_t)s->cap, sizeof(or_lease));
  s->present = (unsigned char*)calloc((size_t)s->cap, 1);
  return s;
}

void or_store_free(or_store* s) {
  if (!s) return;
  free(s->leases);
  free(s->present);
  free(s);
}

static void store_copy_into(or_store* dst, const or_store* src) {
  memcpy(dst->leases, src->leases, (size_t)src->cap * sizeof(or_lease));
  memcpy(dst->present, src->present, (size_t)src->cap);
  dst->sum_wants = src->sum_wants;
  dst->sum_has = src->sum_has;
  dst->count = src->count;
}

or_store* or_store_clone(const or_store* s) {
  or_store* c = or_store_new(s->cap);
  store_copy_into(c, s);
  return c;
}

/* store.go:121-131 Count / SumWants / SumHas */
int64_t or_store_count(const or_store* s) { return s->count; }
double or_store_sum_has(const or_store* s) { return s->sum_has; }
double or_store_sum_wants(const or_store* s) { return s->sum_wants; }

void or_store_set_sums(or_store* s, int64_t count, double sum_has, double sum_wants) {
  s->count = count;
  s->sum_has = sum_has;
  s->sum_wants = sum_wants;
}

/* store.go:133-136 HasClient */
int or_store_has_client(const or_store* s, int64_t client) {
  return client >= 0 && client < s->cap && s->present[client];
}

/* store.go:138-140 Get: the zero Lease when absent */
void or_store_get(const or_store* s, int64_t client, or_lease* out) {
  if (or_store_has_client(s, client))
    *out = s->leases[client];
  else
    memset(out, 0, sizeof(*out));
}

/* store.go:142-151 Release */
void or_store_release(or_store* s, int64_t client) {
  if (!or_store_has_client(s, client)) return;
  const or_lease* l = &s->leases[client];
  s->sum_wants -= l->wants;
  s->sum_has -= l->has;
  s->count -= l->subclients;
  s->present[client] = 0;
  memset(&s->leases[client], 0, sizeof(or_lease));
}

/* store.go:153-167 Assign (time.Now() replaced by the frozen now_ns) */
void or_store_assign(or_store* s, int64_t client, int64_t lease_length_ns, int64_t refresh_ns, double has,
                     double wants, int64_t subclients, int64_t now_ns, or_lease* out) {
  or_lease lease;
  or_store_get(s, client, &lease);
  s->sum_has += has - lease.has;
  s->sum_wants += wants - lease.wants;
  s->count += subclients - lease.subclients;
  lease.has = has;
  lease.wants = wants;
  lease.expiry_ns = now_ns + lease_length_ns;
  lease.refresh_ns = refresh_ns;
  lease.subclients = subclients;
  s->leases[client] = lease;
  s->present[client] = 1;
  if (out) *out = lease;
}

/* Assign-equivalent running-sum update with an explicit stored lease */
void or_store_put(or_store* s, int64_t client, const or_lease* in) {
  or_lease lease;
  or_store_get(s, client, &lease);
  s->sum_has += in->has - lease.has;
  s->sum_wants += in->wants - lease.wants;
  s->count += in->subclients - lease.subclients;
  s->leases[client] = *in;
  s->present[client] = 1;
}

/* store.go:169-181 Clean: release leases with when.After(lease.Expiry) (strict) */
int64_t or_store_clean(or_store* s, int64_t now_ns) {
  int64_t result = 0;
  for (int64_t c = 0; c < s->cap; ++c) {
    if (s->present[c] && now_ns > s->leases[c].expiry_ns) {
      or_store_release(s, c);
      ++result;
    }
  }
  return result;
}

/* ------------------------------------------------------------------------- */
/* algorithm.go                                                               */
/* ------------------------------------------------------------------------- */

/* algorithm.go:50-55 minF (NOT fmin: returns `left` unless left > right) */
static double minF(double left, double right) { return left > right ? right : left; }

/* algorithm.go:46-48 getAlgorithmParams: seconds -> Duration */
static void params(int64_t lease_length_s, int64_t refresh_s, int64_t* len_ns, int64_t* ref_ns) {
  *len_ns = lease_length_s * 1000000000LL;
  *ref_ns = refresh_s * 1000000000LL;
}

/* algorithm.go:95-206 FairShare */
static void fair_share(or_store* s, double capacity, const or_request* r, int64_t len_ns, int64_t ref_ns,
                       int64_t now_ns, or_lease* out) {
  or_lease old;
  or_store_get(s, r->client, &old);                                  /* :102 */
  int64_t count = s->count - old.subclients + r->subclients;         /* :115 */
  double available = capacity - s->sum_has + old.has;                /* :120 */
  double equalShare = capacity / (double)count;                      /* :123 */
  double deservedShare = equalShare * (double)r->subclients;         /* :126 */
  if (r->wants <= deservedShare) {                                   /* :131 */
    or_store_assign(s, r->client, len_ns, ref_ns, minF(r->wants, available), r->wants, r->subclients, now_ns, out);
    return;
  }
  double extra = 0.0;                                                /* :143 */
  int64_t wantExtra = r->subclients;                                 /* :148 */
  int64_t* we = (int64_t*)malloc((size_t)s->cap * sizeof(int64_t)); /* :153 wantExtraClients */
  int64_t nwe = 0;
  for (int64_t id = 0; id < s->cap; ++id) {                          /* :156 store.Map */
    if (!s->present[id]) continue;
    if (id == r->client) continue;                                   /* :157 */
    const or_lease* l = &s->leases[id];
    double deserved = (double)l->subclients * equalShare;            /* :160 */
    if (l->wants < deserved) {
      extra += deserved - l->wants;                                  /* :164 */
    } else if (l->wants > deserved) {
      wantExtra += l->subclients;                                    /* :168 */
      we[nwe++] = id;                                                /* :169 */
    }
  }
  double deservedExtra = (extra / (double)wantExtra) * (double)r->subclients; /* :175 */
  if (r->wants < deservedShare + deservedExtra) {                    /* :179 */
    free(we);
    or_store_assign(s, r->client, len_ns, ref_ns, minF(r->wants, available), r->wants, r->subclients, now_ns, out);
    return;
  }
  int64_t wantExtraExtra = r->subclients;                            /* :189 */
  double extraExtra = 0.0;                                           /* :190 */
  for (int64_t k = 0; k < nwe; ++k) {                                /* :192 */
    int64_t id = we[k];
    if (id == r->client) continue;                                   /* :193 */
    const or_lease* l = &s->leases[id];
    if (l->wants < deservedExtra + deservedShare) {                  /* :197 */
      extraExtra += deservedExtra + deservedShare - l->wants;        /* :198 */
    } else if (l->wants > deservedExtra + deservedShare) {           /* :199 */
      wantExtraExtra += l->subclients;                               /* :200 */
    }
  }
  free(we);
  double deservedExtraExtra = (extraExtra / (double)wantExtraExtra) * (double)r->subclients; /* :203 */
  or_store_assign(s, r->client, len_ns, ref_ns, minF(deservedShare + deservedExtra + deservedExtraExtra, available),
                  r->wants, r->subclients, now_ns, out);             /* :204 */
}

/* algorithm.go:213-293 ProportionalShare */
static void proportional_share(or_store* s, double capacity, const or_request* r, int64_t len_ns, int64_t ref_ns,
                               int64_t now_ns, or_lease* out) {
  int64_t count = s->count;                                          /* :217 */
  or_lease old;
  or_store_get(s, r->client, &old);                                  /* :218 */
  double gets = 0.0;
  if (!or_store_has_client(s, r->client)) count += r->subclients;    /* :223-225 */
  double equalShare = capacity / (double)count;                      /* :229 */
  double equalSharePerClient = equalShare * (double)r->subclients;   /* :233 */
  double unusedCapacity = capacity - s->sum_has + old.has;           /* :239 */
  if (s->sum_wants <= capacity || r->wants <= equalSharePerClient) { /* :245 */
    or_store_assign(s, r->client, len_ns, ref_ns, minF(r->wants, unusedCapacity), r->wants, r->subclients, now_ns,
                    out);
    return;
  }
  double extraCapacity = 0.0, extraNeed = 0.0;                       /* :256-257 */
  for (int64_t id = 0; id < s->cap; ++id) {                          /* :259 store.Map */
    if (!s->present[id]) continue;
    double wants;
    int64_t subclients;
    if (id == r->client) {                                           /* :263-269 */
      wants = r->wants;
      subclients = r->subclients;
    } else {
      wants = s->leases[id].wants;
      subclients = s->leases[id].subclients;
    }
    double esp = equalShare * (double)subclients;                    /* :273 */
    if (wants < esp)
      extraCapacity += esp - wants;                                  /* :275 */
    else
      extraNeed += wants - esp;                                      /* :277 */
  }
  gets = equalSharePerClient + (r->wants - equalSharePerClient) * (extraCapacity / extraNeed); /* :283 */
  or_store_assign(s, r->client, len_ns, ref_ns, minF(gets, unusedCapacity), r->wants, r->subclients, now_ns,
                  out);                                              /* :290 */
}

/* algorithm.go:66-72 NoAlgorithm, :78-84 Static, :297-302 Learn, :304-313 GetAlgorithm */
int or_algorithm(int32_t kind, int64_t lease_length_s, int64_t refresh_interval_s, or_store* s, double capacity,
                 const or_request* r, int64_t now_ns, or_lease* out) {
  int64_t len_ns, ref_ns;
  params(lease_length_s, refresh_interval_s, &len_ns, &ref_ns);
  switch (kind) {
    case OR_NO_ALGORITHM:
      or_store_assign(s, r->client, len_ns, ref_ns, r->wants, r->wants, r->subclients, now_ns, out);
      return 0;
    case OR_STATIC:
      or_store_assign(s, r->client, len_ns, ref_ns, minF(capacity, r->wants), r->wants, r->subclients, now_ns, out);
      return 0;
    case OR_PROPORTIONAL_SHARE:
      proportional_share(s, capacity, r, len_ns, ref_ns, now_ns, out);
      return 0;
    case OR_FAIR_SHARE:
      fair_share(s, capacity, r, len_ns, ref_ns, now_ns, out);
      return 0;
    case OR_LEARN:
      or_store_assign(s, r->client, len_ns, ref_ns, r->has, r->wants, r->subclients, now_ns, out);
      return 0;
    default:
      return -2; /* algorithms[kind] is nil: the reference panics */
  }
}

/* resource.go:62-70 capacity(): 0 after the parent lease expired (expiryTime.Before(now)) */
double or_resource_capacity(const or_resource_cfg* cfg, int64_t now_ns) {
  if (cfg->parent_expiry_ns != INT64_MAX && cfg->parent_expiry_ns < now_ns) return 0.0;
  return cfg->capacity;
}

/* resource.go:100-113 Decide: Clean, then Learn while learningModeEndTime.After(now), else the algorithm */
int or_decide(or_store* s, const or_resource_cfg* cfg, const or_request* r, int64_t now_ns, or_lease* out) {
  if (cfg->kind < OR_NO_ALGORITHM || cfg->kind > OR_FAIR_SHARE) return -2;
  or_store_clean(s, now_ns);
  if (cfg->learning_end_ns > now_ns)
    return or_algorithm(OR_LEARN, cfg->lease_length_s, cfg->refresh_interval_s, s, or_resource_capacity(cfg, now_ns),
                        r, now_ns, out);
  return or_algorithm(cfg->kind, cfg->lease_length_s, cfg->refresh_interval_s, s, or_resource_capacity(cfg, now_ns), r,
                      now_ns, out);
}

/* server.go:850-868 band aggregation of GetServerCapacity */
int or_aggregate_bands(const double* wants, const int64_t* num_clients, int64_t n, double* wants_total,
                       int64_t* subclients_total) {
  double wt = 0.0;
  int64_t st = 0;
  for (int64_t i = 0; i < n; ++i) {
    wt += wants[i];
    if (num_clients[i] < 1) return -1;
    st += num_clients[i];
  }
  *wants_total = wt;
  *subclients_total = st;
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Snapshot batch                                                             */
/* ------------------------------------------------------------------------- */

/* Materialise resource r of the snapshot as a Go store: one Assign per row in
 * row order (running sums, store.go:156-158), the parity-mode sums if given,
 * then Clean (store.go:169-181). */
static or_store* build_store(const or_snapshot* sn, int64_t r, int64_t now_ns) {
  int64_t lo = sn->seg_off[r], hi = sn->seg_off[r + 1];
  or_store* s = or_store_new(hi - lo);
  for (int64_t i = lo; i < hi; ++i) {
    or_lease l;
    l.expiry_ns = sn->expiry_ns[i];
    l.refresh_ns = sn->cfg[r].refresh_interval_s * 1000000000LL;
    l.has = sn->has[i];
    l.wants = sn->wants[i];
    l.subclients = sn->subclients[i];
    or_store_put(s, i - lo, &l);
  }
  if (sn->agg_count) or_store_set_sums(s, sn->agg_count[r], sn->agg_sum_has[r], sn->agg_sum_wants[r]);
  or_store_clean(s, now_ns);
  return s;
}

static void finish_resource(const or_snapshot* sn, int64_t r, int64_t count, double sum_has_clean,
                            double sum_wants_clean, const double* gets, const int64_t* expiry, or_outputs* out) {
  int64_t lo = sn->seg_off[r], hi = sn->seg_off[r + 1];
  /* the tick's Assigns, applied in row order: sumHas += gets - has (store.go:156) */
  double sh = sum_has_clean;
  for (int64_t i = lo; i < hi; ++i)
    if (expiry[i] != OR_RELEASED) sh += gets[i] - sn->has[i];
  if (out->res_count) out->res_count[r] = count;
  if (out->res_sum_has) out->res_sum_has[r] = sh;
  if (out->res_sum_wants) out->res_sum_wants[r] = sum_wants_clean;
  if (out->res_safe_capacity) {
    /* resource.go:91-95 SetSafeCapacity */
    double safe = sn->cfg[r].safe_capacity;
    out->res_safe_capacity[r] = isnan(safe) ? sn->cfg[r].capacity / (double)count : safe;
  }
}

/* Literal snapshot semantics: every row is a request (has, wants, subclients
 * from the row) decided by Resource.Decide on a private clone of the frozen
 * store.  Rows that Clean releases get no lease (OR_RELEASED). */
int or_apportion_literal(const or_snapshot* sn, int64_t now_ns, or_outputs* out) {
  for (int64_t r = 0; r < sn->n_resources; ++r)
    if (sn->cfg[r].kind < OR_NO_ALGORITHM || sn->cfg[r].kind > OR_FAIR_SHARE) return -2;
  for (int64_t r = 0; r < sn->n_resources; ++r) {
    int64_t lo = sn->seg_off[r], hi = sn->seg_off[r + 1];
    or_store* base = build_store(sn, r, now_ns);
    or_store* work = or_store_new(hi - lo);
    for (int64_t i = lo; i < hi; ++i) {
      if (!base->present[i - lo]) {
        out->gets[i] = 0.0;
        out->expiry_ns[i] = OR_RELEASED;
        continue;
      }
      store_copy_into(work, base);
      or_request q = {i - lo, sn->has[i], sn->wants[i], sn->subclients[i]};
      or_lease l;
      or_decide(work, &sn->cfg[r], &q, now_ns, &l);
      out->gets[i] = l.has;
      out->expiry_ns[i] = l.expiry_ns;
    }
    finish_resource(sn, r, base->count, base->sum_has, base->sum_wants, out->gets, out->expiry_ns, out);
    or_store_free(work);
    or_store_free(base);
  }
  return 0;
}

int64_t or_apportion_literal_rows(const or_snapshot* sn, int64_t r, int64_t row_lo, int64_t row_hi, int64_t now_ns,
                                  double* gets) {
  int64_t lo = sn->seg_off[r], hi = sn->seg_off[r + 1];
  if (row_lo < lo) row_lo = lo;
  if (row_hi > hi) row_hi = hi;
  or_store* base = build_store(sn, r, now_ns);
  or_store* work = or_store_new(hi - lo);
  int64_t n = 0;
  for (int64_t i = row_lo; i < row_hi; ++i) {
    if (!base->present[i - lo]) continue;
    store_copy_into(work, base);
    or_request q = {i - lo, sn->has[i], sn->wants[i], sn->subclients[i]};
    or_lease l;
    or_decide(work, &sn->cfg[r], &q, now_ns, &l);
    gets[i] = l.has;
    ++n;
  }
  or_store_free(work);
  or_store_free(base);
  return n;
}

/* or_apportion_literal_rows over a list of resources on `threads` OpenMP threads
 * (rows [lo, lo + row_cap) of each): the reference's per-request Decide timed at
 * the host's width (bench.py cpu_baseline). */
int64_t or_apportion_literal_sample(const or_snapshot* sn, const int64_t* res, int64_t nres, int64_t row_cap,
                                    int64_t now_ns, double* gets, int threads) {
  int64_t total = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1) reduction(+ : total)
  for (int64_t k = 0; k < nres; ++k) {
    const int64_t r = res[k], lo = sn->seg_off[r];
    total += or_apportion_literal_rows(sn, r, lo, lo + row_cap, now_ns, gets);
  }
  return total;
}

/* Closed form with every sum taken in row order, which makes
 * it bit-identical to or_apportion_literal. */
typedef struct {
  double T;
  double ee;
  int64_t sgt;
} t_entry;

/* One resource of the closed form; *cache / *cache_cap: the caller's scratch for
 * distinct round-2 thresholds (one per thread in the threaded variant). */
static void closed_resource(const or_snapshot* sn, int64_t r, int64_t now_ns, or_outputs* out, t_entry** cache_p,
                            int64_t* cache_cap_p) {
  t_entry* cache = *cache_p;
  int64_t cache_cap = *cache_cap_p;
  {
    const or_resource_cfg* cfg = &sn->cfg[r];
    int64_t lo = sn->seg_off[r], hi = sn->seg_off[r + 1];
    /* store sums: Assign per row in order, parity override, Clean in order */
    int64_t count = 0;
    double sum_has = 0.0, sum_wants = 0.0;
    for (int64_t i = lo; i < hi; ++i) {
      sum_has += sn->has[i] - 0.0;
      sum_wants += sn->wants[i] - 0.0;
      count += sn->subclients[i] - 0;
    }
    if (sn->agg_count) {
      count = sn->agg_count[r];
      sum_has = sn->agg_sum_has[r];
      sum_wants = sn->agg_sum_wants[r];
    }
    for (int64_t i = lo; i < hi; ++i) {
      if (now_ns > sn->expiry_ns[i]) {
        sum_wants -= sn->wants[i];
        sum_has -= sn->has[i];
        count -= sn->subclients[i];
      }
    }
    const double C = or_resource_capacity(cfg, now_ns);
    const int learning = cfg->learning_end_ns > now_ns;
    const int64_t len_ns = cfg->lease_length_s * 1000000000LL;
    const double eq = C / (double)count;
    double E = 0.0, xc = 0.0, xn = 0.0;
    int64_t W = 0;
    if (!learning && (cfg->kind == OR_FAIR_SHARE || cfg->kind == OR_PROPORTIONAL_SHARE)) {
      for (int64_t j = lo; j < hi; ++j) {
        if (now_ns > sn->expiry_ns[j]) continue;
        double w = sn->wants[j];
        int64_t sj = sn->subclients[j];
        if (cfg->kind == OR_FAIR_SHARE) {
          double d = (double)sj * eq;
          if (w < d)
            E += d - w;
          else if (w > d)
            W += sj;
        } else {
          double e = eq * (double)sj;
          if (w < e)
            xc += e - w;
          else
            xn += w - e;
        }
      }
    }
    int64_t ncache = 0;
    for (int64_t i = lo; i < hi; ++i) {
      if (now_ns > sn->expiry_ns[i]) {
        out->gets[i] = 0.0;
        out->expiry_ns[i] = OR_RELEASED;
        continue;
      }
      out->expiry_ns[i] = now_ns + len_ns;
      const double w = sn->wants[i], h = sn->has[i];
      const int64_t si = sn->subclients[i];
      double g;
      if (learning) {
        g = h;
      } else if (cfg->kind == OR_NO_ALGORITHM) {
        g = w;
      } else if (cfg->kind == OR_STATIC) {
        g = minF(C, w);
      } else if (cfg->kind == OR_PROPORTIONAL_SHARE) {
        double epc = eq * (double)si;
        double unused = C - sum_has + h;
        if (sum_wants <= C || w <= epc)
          g = minF(w, unused);
        else
          g = minF(epc + (w - epc) * (xc / xn), unused);
      } else { /* FAIR_SHARE */
        double ds = eq * (double)si;
        double avail = C - sum_has + h;
        if (w <= ds) {
          g = minF(w, avail);
        } else {
          int64_t Wi = W + si - (w > ds ? si : 0);
          double dE = (E / (double)Wi) * (double)si;
          if (w < ds + dE) {
            g = minF(w, avail);
          } else {
            double T = dE + ds;
            t_entry* hit = NULL;
            for (int64_t k = 0; k < ncache; ++k)
              if (memcmp(&cache[k].T, &T, sizeof(double)) == 0) {
                hit = &cache[k];
                break;
              }
            if (!hit) {
              if (ncache == cache_cap) {
                cache_cap = cache_cap ? 2 * cache_cap : 16;
                cache = (t_entry*)realloc(cache, (size_t)cache_cap * sizeof(t_entry));
              }
              hit = &cache[ncache++];
              hit->T = T;
              hit->ee = 0.0;
              hit->sgt = 0;
              for (int64_t j = lo; j < hi; ++j) {
                if (now_ns > sn->expiry_ns[j]) continue;
                double wj = sn->wants[j];
                int64_t sj = sn->subclients[j];
                double dj = (double)sj * eq;
                if (!(wj > dj)) continue; /* j in wantExtraClients */
                if (wj < T)
                  hit->ee += T - wj;
                else if (wj > T)
                  hit->sgt += sj;
              }
            }
            int64_t wee = si + hit->sgt - ((w > ds && w > T) ? si : 0);
            double dEE = (hit->ee / (double)wee) * (double)si;
            g = minF(ds + dE + dEE, avail);
          }
        }
      }
      out->gets[i] = g;
    }
    finish_resource(sn, r, count, sum_has, sum_wants, out->gets, out->expiry_ns, out);
  }
  *cache_p = cache;
  *cache_cap_p = cache_cap;
}

static int check_kinds(const or_snapshot* sn) {
  for (int64_t r = 0; r < sn->n_resources; ++r)
    if (sn->cfg[r].kind < OR_NO_ALGORITHM || sn->cfg[r].kind > OR_FAIR_SHARE) return -2;
  return 0;
}

int or_apportion_closed(const or_snapshot* sn, int64_t now_ns, or_outputs* out) {
  if (check_kinds(sn)) return -2;
  t_entry* cache = NULL;
  int64_t cache_cap = 0;
  for (int64_t r = 0; r < sn->n_resources; ++r) closed_resource(sn, r, now_ns, out, &cache, &cache_cap);
  free(cache);
  return 0;
}

/* The closed form over resources in parallel (OpenMP, `threads` threads): the
 * optimised-CPU comparator of SURVEY.md §8(d)(iii).  Resources are independent,
 * so the outputs are identical to or_apportion_closed. */
int or_apportion_closed_mt(const or_snapshot* sn, int64_t now_ns, or_outputs* out, int threads) {
  if (check_kinds(sn)) return -2;
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
  {
    t_entry* cache = NULL;
    int64_t cache_cap = 0;
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = 0; r < sn->n_resources; ++r) closed_resource(sn, r, now_ns, out, &cache, &cache_cap);
    free(cache);
  }
  return 0;
}
