/*
 * doorman_oracle.h — CPU restatement of Doorman's lease algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (doorman_amd/, include/,
 * the C-ABI library) includes, links or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline.
 *
 * Parity status: PINNED.  Every expectation in the reference's own tests
 * (go/server/doorman/algorithm_test.go:274-522, store_test.go:22-77,
 * server_test.go:339-553) and the worked examples in doc/algorithms.md:47-67 and
 * doc/simplecluster/README.md:271-296,411-435 are replayed against this code by
 * tests/test_oracle_golden.py from tests/golden/reference_kats.json.
 *
 * Two evaluators are provided:
 *   - "literal":  go/server/doorman/store.go + algorithm.go + resource.go restated
 *                 statement by statement (Go map iteration replaced by ascending
 *                 client-id order: Go's order is random, so any fixed order is a
 *                 valid reference execution).
 *   - "closed":   the per-resource closed form of SURVEY.md §8(a), summing in row
 *                 order; bit-identical to "literal" in snapshot mode.
 *
 * Go float64 == IEEE-754 binary64, round-to-nearest, no FMA contraction on amd64:
 * compile with -ffp-contract=off -fno-fast-math (oracle/Makefile does).
 */
#ifndef DOORMAN_ORACLE_H
#define DOORMAN_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* pb.Algorithm_Kind, proto/doorman/doorman.proto:139-144 */
enum {
  OR_NO_ALGORITHM = 0,
  OR_STATIC = 1,
  OR_PROPORTIONAL_SHARE = 2,
  OR_FAIR_SHARE = 3,
  OR_LEARN = 4 /* algorithm.go:297 Learn (not a proto kind; used internally) */
};

#define OR_RELEASED INT64_MIN /* expiry marker for a row released by Clean */

/* store.go:20-36 Lease (times as int64 unix nanoseconds) */
typedef struct {
  int64_t expiry_ns;  /* 0 == zero time.Time (IsZero) */
  int64_t refresh_ns;
  double has;
  double wants;
  int64_t subclients;
} or_lease;

/* algorithm.go:27-40 Request (Client is a dense id) */
typedef struct {
  int64_t client;
  double has;
  double wants;
  int64_t subclients;
} or_request;

/* resolved per-resource configuration (resource.go:37-57, doorman.proto:147-190) */
typedef struct {
  int32_t kind;
  double capacity;
  int64_t lease_length_s;
  int64_t refresh_interval_s;
  int64_t learning_end_ns;  /* learningModeEndTime (resource.go:153-163) */
  int64_t parent_expiry_ns; /* Resource.expiryTime; INT64_MAX == nil */
  double safe_capacity;     /* NaN == unset (resource.go:91) */
} or_resource_cfg;

typedef struct or_store or_store;

/* ---- store.go ---- */
or_store* or_store_new(int64_t max_clients);
void or_store_free(or_store* s);
or_store* or_store_clone(const or_store* s);
int64_t or_store_count(const or_store* s);
double or_store_sum_has(const or_store* s);
double or_store_sum_wants(const or_store* s);
void or_store_set_sums(or_store* s, int64_t count, double sum_has, double sum_wants);
int or_store_has_client(const or_store* s, int64_t client);
void or_store_get(const or_store* s, int64_t client, or_lease* out);
void or_store_release(or_store* s, int64_t client);
void or_store_assign(or_store* s, int64_t client, int64_t lease_length_ns, int64_t refresh_ns, double has,
                     double wants, int64_t subclients, int64_t now_ns, or_lease* out);
/* Assign with an explicit expiry (used to materialise a snapshot row) */
void or_store_put(or_store* s, int64_t client, const or_lease* lease);
int64_t or_store_clean(or_store* s, int64_t now_ns);

/* ---- algorithm.go ---- */
int or_algorithm(int32_t kind, int64_t lease_length_s, int64_t refresh_interval_s, or_store* s, double capacity,
                 const or_request* r, int64_t now_ns, or_lease* out);

/* ---- resource.go:62-70 capacity(), :100-113 Decide ---- */
double or_resource_capacity(const or_resource_cfg* cfg, int64_t now_ns);
int or_decide(or_store* s, const or_resource_cfg* cfg, const or_request* r, int64_t now_ns, or_lease* out);

/* ---- server.go:850-879 GetServerCapacity band aggregation ----
 * returns 0, or -1 (codes.InvalidArgument) when some num_clients < 1 */
int or_aggregate_bands(const double* wants, const int64_t* num_clients, int64_t n, double* wants_total,
                       int64_t* subclients_total);

/* ---- snapshot batch ----
 * Snapshot of R resources, CSR segments seg_off[R+1] over N lease rows.
 * agg_* may be NULL (store sums rebuilt from the rows by sequential Assign) or
 * give the store's running sums (parity mode).
 * Outputs: gets[N], expiry_ns[N] (OR_RELEASED for rows Clean drops);
 * per resource: count/sum_has/sum_wants after the tick, safe capacity.
 * Returns 0, or -2 for an unknown algorithm kind (the reference panics). */
typedef struct {
  int64_t n_resources;
  int64_t n_leases;
  const int64_t* seg_off;
  const double* wants;
  const double* has;
  const int64_t* subclients;
  const int64_t* expiry_ns;
  const or_resource_cfg* cfg;
  const int64_t* agg_count;
  const double* agg_sum_has;
  const double* agg_sum_wants;
} or_snapshot;

typedef struct {
  double* gets;
  int64_t* expiry_ns;
  int64_t* res_count;
  double* res_sum_has;
  double* res_sum_wants;
  double* res_safe_capacity;
} or_outputs;

int or_apportion_literal(const or_snapshot* snap, int64_t now_ns, or_outputs* out);
int or_apportion_closed(const or_snapshot* snap, int64_t now_ns, or_outputs* out);
/* Same outputs, resources spread over `threads` OpenMP threads. */
int or_apportion_closed_mt(const or_snapshot* snap, int64_t now_ns, or_outputs* out, int threads);

/* literal evaluation restricted to rows [row_lo,row_hi) of one resource
 * (bounded CPU-baseline samples); returns number of rows evaluated */
int64_t or_apportion_literal_rows(const or_snapshot* snap, int64_t resource, int64_t row_lo, int64_t row_hi,
                                  int64_t now_ns, double* gets);
/* the same over nres resources (rows [lo, lo + row_cap) of each) on `threads`
 * OpenMP threads; returns the number of rows evaluated */
int64_t or_apportion_literal_sample(const or_snapshot* snap, const int64_t* resources, int64_t nres, int64_t row_cap,
                                    int64_t now_ns, double* gets, int threads);

#ifdef __cplusplus
}
#endif
#endif
