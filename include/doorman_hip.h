/*
 * doorman_hip.h — C-ABI of the MI355X batched lease-apportionment engine.
 *
 * Drop-in boundary for Doorman's lease path (paths relative to the reference
 * repository root).  The reference binds no native code; these entry points are
 * what a cgo shim behind its own interfaces would call (INTEGRATION.md shows the
 * Go side):
 *
 *   LeaseStore interface        go/server/doorman/store.go:68-103   -> dm_store_* / dm_read_*
 *   NewLeaseStore               go/server/doorman/store.go:114      -> dm_create + dm_store_load
 *   Algorithm (per request)     go/server/doorman/algorithm.go:44   -> dm_apportion (batch of every client)
 *   GetAlgorithm / algorithms   go/server/doorman/algorithm.go:304-313 -> dm_resource_cfg.kind
 *   Resource.Decide             go/server/doorman/resource.go:100-113  -> dm_apportion (Clean + learning + algorithm)
 *   Resource.capacity           go/server/doorman/resource.go:62-70    -> dm_resource_cfg.parent_expiry_ns
 *   Resource.SetSafeCapacity    go/server/doorman/resource.go:81-96    -> dm_read_resources(.safe_capacity)
 *   GetCapacity lease -> proto  go/server/doorman/server.go:787-791    -> dm_read_leases (unix seconds)
 *   performRequests aggregation go/server/doorman/server.go:234-255    -> dm_read_resources(count, sum_wants)
 *   GetServerCapacity bands     go/server/doorman/server.go:850-879    -> dm_aggregate_bands
 *
 * Batch semantics: every stored lease row is also that client's refresh request
 * (has, wants, subclients taken from the row) and is decided against the same
 * frozen store, as if Resource.Decide ran on a private copy of the store for
 * each client at time now_ns.  Rows that Clean drops (now_ns > expiry_ns,
 * store.go:174) are released and get no lease (expiry DM_RELEASED).
 *
 * Conventions: plain pointers and sizes only; every host pointer is read or
 * written before the call returns (the caller keeps ownership); return 0 on
 * success or a negative DM_E_* code, with a message in dm_last_error(ctx).
 * One call in flight per context; different contexts (GPUs) are independent.
 */
#ifndef DOORMAN_HIP_H
#define DOORMAN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 6 (round 6): dm_store_apply_async / dm_store_apply_wait (a round's store batch enqueued
   without waiting; its outcome reported by a later call).
   5 (round 6): dm_store_lost (the read calls work on a lost store); dm_plan_info's slot 18 is the class streams' hardware-queue assignment the
   context's queue calibration chose (-1 before it finished); returns 19.
   4 (round 5): dm_kernel_class_names, dm_hier_comm_info; dm_plan_info's slot 14 is the
   redo's co-resident workgroup bound (was the per-chunk redo's chunk bound), slot 15
   always 1, slot 16 the aux queues flag, slot 17 the stream parts; a published block's
   record 0 holds two 32-bit flags words (their OR is the request's flags); the DM_*
   environment switches other than the test hooks are gone.  3 (round 4): dm_hier_attach / dm_hier_step / dm_rccl_unique_id /
   dm_hier_comm_init and DM_E_INTERNAL added, dm_set_large_path and DM_LARGE_* removed. */
#define DM_ABI_VERSION 6

/* return codes */
#define DM_OK 0
#define DM_E_INVAL (-1)   /* bad argument / shape */
#define DM_E_HIP (-2)     /* HIP runtime failure (message has the HIP error) */
#define DM_E_STATE (-3)   /* no store / config loaded, or sizes disagree */
#define DM_E_KIND (-4)    /* unknown algorithm kind (the reference panics: algorithm.go:312) */
#define DM_E_RANGE (-5)   /* row / resource index out of range */
#define DM_E_ARGUMENT (-6) /* codes.InvalidArgument, e.g. num_clients < 1 (server.go:863-866) */
#define DM_E_INTERNAL (-7) /* an internal invariant failed (a bug in this library) */

/* pb.Algorithm_Kind (proto/doorman/doorman.proto:139-144) */
#define DM_NO_ALGORITHM 0
#define DM_STATIC 1
#define DM_PROPORTIONAL_SHARE 2
#define DM_FAIR_SHARE 3

#define DM_RELEASED INT64_MIN /* expiry of a lease Clean released (store.go:169-181) */
#define DM_NO_PARENT_EXPIRY INT64_MAX /* Resource.expiryTime == nil (resource.go:64) */
#define DM_NO_LEARNING INT64_MIN      /* learning mode disabled (server.go:173-179) */

/* dm_apportion flags */
#define DM_WRITEBACK 1u     /* store the tick: has := gets, expiry := lease expiry, released rows zeroed,
                               running sums updated as the Assigns would (store.go:153-167) */
#define DM_AGG_RECOMPUTE 2u /* ignore the store's running sums; recompute them from the rows */
#define DM_ASYNC 4u         /* enqueue on the context stream and return without waiting */
/* Where a writeback tick writes gets/expiry.  Default: in place for a store that
   fits the Infinity Cache, else into a second pair of has/expiry columns that
   becomes the store's after the tick (faster streaming; 16 B per lease of HBM). */
#define DM_WB_INPLACE 8u    /* force in-place writeback */
#define DM_WB_ALTERNATE 16u /* force the alternate columns */
#define DM_DEFER_JOIN 32u   /* with DM_ASYNC: a tick whose work classes run on the context's
                               auxiliary streams need not join them back into the context
                               stream at its end.  Every later library call on the context
                               joins first; work the caller itself puts on the context
                               stream is ordered after the tick only after dm_join or
                               dm_sync.  Back-to-back ticks then skip two cross-queue hops
                               each (C2: 240 -> 191 us per tick). */

typedef struct dm_ctx dm_ctx;

/* Frozen store snapshot: R resources as CSR segments over N lease rows (SoA). */
typedef struct {
  int64_t n_resources;
  int64_t n_leases;
  const int64_t* seg_off;    /* [R+1] resource r owns rows [seg_off[r], seg_off[r+1]) */
  const double* wants;       /* [N] Lease.Wants */
  const double* has;         /* [N] Lease.Has */
  const int64_t* subclients; /* [N] Lease.Subclients, 0 <= v < 2^31 - 1 (DM_E_INVAL otherwise) */
  const int64_t* expiry_ns;  /* [N] Lease.Expiry, unix ns */
  const int64_t* agg_count;  /* [R] or NULL: store.count     (running sum; NULL = recompute) */
  const double* agg_sum_has; /* [R] or NULL: store.sumHas */
  const double* agg_sum_wants; /* [R] or NULL: store.sumWants */
} dm_snapshot;

/* Resolved per-resource configuration, SoA over R resources. */
typedef struct {
  const int32_t* kind;              /* DM_* algorithm kind */
  const double* capacity;           /* ResourceTemplate.capacity */
  const int64_t* lease_length_s;    /* Algorithm.lease_length, seconds in [0, 2^31) (DM_E_INVAL otherwise) */
  const int64_t* refresh_interval_s; /* Algorithm.refresh_interval, seconds in [0, 2^31) */
  const int64_t* learning_end_ns;   /* learningModeEndTime; DM_NO_LEARNING = none */
  const int64_t* parent_expiry_ns;  /* parent lease expiry; DM_NO_PARENT_EXPIRY = nil */
  const double* safe_capacity;      /* ResourceTemplate.safe_capacity; NaN = unset */
} dm_resource_cfg;

/* One round of store updates (dm_store_apply): the parts are applied in this order,
   each exactly as the single call named beside it; a part with n == 0 (or
   wants_nwords == 0) is skipped.  All parts' columns cross PCIe back to back on the
   copy stream, so a part's validation and apply overlap the later parts' copies. */
typedef struct {
  /* refresh of existing clients' wants (dm_store_update_wants_mask) */
  int64_t wants_first_row, wants_nwords;
  const uint64_t* wants_mask;
  int64_t wants_n;
  const double* wants;
  /* departures (dm_store_release) */
  int64_t release_n;
  const int64_t* release_rows;
  /* arrivals and full refreshes (dm_store_upsert) */
  int64_t upsert_n;
  const int64_t* upsert_rows;
  const double* upsert_has;          /* NULL: 0 for every row (a new client holds nothing yet) */
  const double* upsert_wants;
  const int64_t* upsert_subclients;  /* or NULL with upsert_subclients32 */
  const int64_t* upsert_expiry_ns;   /* NULL: each row's resource's upsert_now_ns + lease length (the
                                        expiry Assign gives, store.go:161) */
  /* narrow arrivals: 4-B subclients instead of upsert_subclients (C4's arrivals: 20 B per
     row over PCIe with has and expiry NULL, instead of 40) */
  const int32_t* upsert_subclients32;
  int64_t upsert_now_ns;             /* required (> 0, else DM_E_INVAL) when upsert_expiry_ns is NULL */
} dm_store_batch;

typedef struct {
  const char* name;
  int64_t launches;
  double total_ms; /* HIP-event time summed over launches (profiling on) */
} dm_kernel_time;

/* ---- context ---- */
const char* dm_version(void);
int dm_device_count(int* out);
int dm_create(int device, dm_ctx** out);
void dm_destroy(dm_ctx* ctx);
const char* dm_last_error(dm_ctx* ctx);
/* use an existing hipStream_t (e.g. the caller's current stream); NULL = the context's own.
   The HIP null stream therefore cannot be selected: a caller whose current stream is the
   null stream (torch's default) must create a stream to share (doorman_amd/hierarchy.py). */
int dm_set_stream(dm_ctx* ctx, void* hip_stream);
/* The context stream.  After dm_destroy the handle must not be used: the stream stays
   alive (the library pools a destroyed context's streams for the next context on the
   device), so work queued on it would run in another context's stream. */
void* dm_get_stream(dm_ctx* ctx);
int dm_sync(dm_ctx* ctx);
/* Order every deferred tick (DM_DEFER_JOIN) before later work on the context stream,
   without waiting on the host. */
int dm_join(dm_ctx* ctx);
/* Order hip_stream (any stream of the context's device, e.g. a collective's) after the
   work enqueued so far on the context, deferred tick work included, without waiting on
   the host: a stream memory write on the context stream and a wait for it on
   hip_stream.  An event record + hipStreamWaitEvent does the same at several times the
   GPU-side latency per hop.  Used by the pipelined hierarchy before its
   all-gather (doorman_amd/hierarchy.py). */
int dm_stream_wait(dm_ctx* ctx, void* hip_stream);

/* ---- LeaseStore: device-resident columnar table ---- */
int dm_store_load(dm_ctx* ctx, const dm_snapshot* snap);
int dm_config_load(dm_ctx* ctx, int64_t n_resources, const dm_resource_cfg* cfg);
/* Assign (store.go:153-167) on existing rows: sums += new - old; expiry_ns as given */
int dm_store_upsert(dm_ctx* ctx, int64_t n, const int64_t* rows, const double* has, const double* wants,
                    const int64_t* subclients, const int64_t* expiry_ns);
/* Assign of a refresh that only changes wants (store.go:153-167 with has, subclients and
 * expiry unchanged): sumWants += new - old.  12 bytes per update over PCIe.  A released
 * row is a free slot, not a client: a refresh naming it changes nothing (a returning
 * client is an arrival: dm_store_upsert).  The same holds for the mask form below. */
int dm_store_update_wants(dm_ctx* ctx, int64_t n, const int64_t* rows, const double* wants);
/* The same narrow Assign with the rows given as a bit mask: bit j of mask[w] is row
   first_row + 64*w + j (first_row a multiple of 64); the n set rows take wants[0..n)
   in ascending row order.  Smaller than row indices above ~3% of the rows (C4's 10%
   wants refresh: 116 instead of 200 MB over PCIe).  DM_E_RANGE for a bit past the
   store's end, DM_E_INVAL when n differs from the mask's popcount; a rejected call
   leaves the store untouched. */
int dm_store_update_wants_mask(dm_ctx* ctx, int64_t first_row, int64_t nwords, const uint64_t* mask, int64_t n,
                               const double* wants);
/* Release (store.go:142-151): sums -= row; row zeroed and marked DM_RELEASED.  A released
 * row is a free slot: dm_store_upsert onto it is Assign of a new client. */
int dm_store_release(dm_ctx* ctx, int64_t n, const int64_t* rows);
/* The three update kinds of one round in one call (see dm_store_batch).  Parts run
   in order; the first rejected part returns its error, earlier parts stay applied
   and later ones are not applied.  Synchronous on return, like the single calls. */
int dm_store_apply(dm_ctx* ctx, const dm_store_batch* batch);
/* dm_store_apply without waiting: the batch's copies and kernels are enqueued (ordered
   after the context's earlier work, before its later ticks) and the call returns.  The
   batch's host columns must stay unchanged until the batch is retired: by
   dm_store_apply_wait, or by the dm_store_apply_async call two batches later, which
   first waits for it (so the host runs at most two batches ahead of the device).  A
   retired batch that was rejected fails that retiring call (DM_E_RANGE / DM_E_INVAL,
   the message naming "an earlier asynchronous batch" and its part), and the retiring
   dm_store_apply_async then enqueues nothing; as with dm_store_apply, the rejected part
   and the batch's later parts are not applied, its earlier parts are, and so is every
   batch enqueued after it.  While a batch with a refresh or arrivals is in flight, ticks
   are prepared for heterogeneous subclients (k_general) as for a maybe-general store.
   dm_store_load and dm_config_load wait for in-flight batches first (their outcome is
   dropped).  The C4 streaming round: its PCIe copies back to back from round to round
   (DESIGN.md §5). */
int dm_store_apply_async(dm_ctx* ctx, const dm_store_batch* batch);
/* Retire every in-flight dm_store_apply_async batch, oldest first; returns the first
   failure (DM_OK if none). */
int dm_store_apply_wait(dm_ctx* ctx);
/* The three update calls validate on the device (rows in [0, N), unique within the
 * call, subclients in [0, 2^31 - 1)); a rejected call (DM_E_RANGE / DM_E_INVAL) leaves the
 * store untouched.  They return after the update is applied, so the caller may reuse
 * its buffers.  Buffers from dm_host_alloc (page-locked) go over PCIe by DMA at full
 * rate; ordinary host memory is staged by the HIP runtime. */
int dm_host_alloc(dm_ctx* ctx, size_t bytes, void** out);
int dm_host_free(dm_ctx* ctx, void* ptr);
/* Whether a device-side invariant failed (a redo workgroup gave up, a dense kernel queued
 * an item a skipped launch would have decided): *lost = 1, with the reason in
 * dm_last_error.  A lost store refuses ticks and updates (DM_E_INTERNAL) until
 * dm_store_load; the read calls below still work on it, so its state can be inspected. */
int dm_store_lost(dm_ctx* ctx, int* lost);
/* read back stored rows (has/wants/subclients/expiry_ns) — any pointer may be NULL */
int dm_read_store(dm_ctx* ctx, int64_t off, int64_t n, double* has, double* wants, int64_t* subclients,
                  int64_t* expiry_ns);

/* the resolved configuration the device holds for resources [r0, r0+n) (the
 * dm_resource_cfg columns; Resource.config / Status, resource.go:190-203) -- after a
 * hierarchy exchange, the templates dm_hier_root_tick loaded; any pointer may be NULL */
int dm_read_config(dm_ctx* ctx, int64_t r0, int64_t n, int32_t* kind, double* capacity, int64_t* lease_length_s,
                   int64_t* refresh_interval_s, int64_t* learning_end_ns, int64_t* parent_expiry_ns,
                   double* safe_capacity);

/* ---- the batch algorithm: every client of every resource, one frozen snapshot ---- */
int dm_apportion(dm_ctx* ctx, int64_t now_ns, uint32_t flags);

/* A round of individual requests (Resource.Decide, resource.go:100-113, for each):
 * request k is for the client whose lease lives in row rows[k] -- its existing row,
 * or a free (released) row of the resource it asks for, which makes it a new client
 * (store.HasClient false, algorithm.go:223-225).  After a Clean at now_ns (not
 * written back), the requests are decided in the order given, as res.mu serialises
 * the reference's calls (resource.go:103-104): each with the request's own has
 * (Learn), wants and subclients for its client and the rows for everyone else
 * (algorithm.go:115,126,148,157,263-269), and each decision's Assign (store.go:
 * 153-167: the row and the running sums) is seen by the later requests on the same
 * resource -- so a round's grants stay within the capacity exactly as the
 * reference's.  A row may be requested more than once (a client's later request
 * sees its earlier one).  gets[k] and expiry_ns[k] (now + lease length) are the
 * leases; the device store is not changed -- Assign the final ones with
 * dm_store_upsert.  Subclients in [0, 2^31 - 1).  Synchronous. */
int dm_decide(dm_ctx* ctx, int64_t now_ns, int64_t n, const int64_t* rows, const double* has, const double* wants,
              const int64_t* subclients, double* gets, int64_t* expiry_ns);

/* lease outputs of the last dm_apportion: gets (Lease.Has), expiry in unix ns
 * (DM_RELEASED for released rows); any pointer may be NULL */
int dm_read_leases(dm_ctx* ctx, int64_t off, int64_t n, double* gets, int64_t* expiry_ns);
/* the same for n scattered rows (gathered on the device) */
int dm_read_leases_rows(dm_ctx* ctx, int64_t n, const int64_t* rows, double* gets, int64_t* expiry_ns);
/* proto form (server.go:787-791): capacity, expiry_time = Expiry.Unix(), refresh_interval seconds */
int dm_read_leases_proto(dm_ctx* ctx, int64_t off, int64_t n, double* capacity, int64_t* expiry_time_s,
                         int64_t* refresh_interval_s);
/* per-resource results of the last dm_apportion: store Count/SumHas/SumWants after
 * the tick, and the safe capacity SetSafeCapacity would report */
int dm_read_resources(dm_ctx* ctx, int64_t r0, int64_t n, int64_t* count, double* sum_has, double* sum_wants,
                      double* safe_capacity);

/* ---- hierarchy (intermediate servers) ---- */
/* server.go:850-879: wants_total = sum(wants), subclients_total = sum(num_clients);
 * DM_E_ARGUMENT when some num_clients < 1 */
int dm_aggregate_bands(const double* wants, const int64_t* num_clients, int64_t n, double* wants_total,
                       int64_t* subclients_total);
/* server.go:234-255: what this intermediate server sends upstream, into a device buffer
 * of 1 + R records of 16 B, ready for an RCCL all-gather: record 1 + r = {SumWants f64,
 * Count i64} of resource r (the root sees a band where SumWants > 0, :241); record 0 =
 * {the request's validation flags as int64 bits, 0}: DM_HIER_INVALID when some band has
 * Count < 1 (the root fails the whole GetServerCapacity, :863-866), DM_HIER_COUNT_RANGE
 * when a Count does not fit the root's 32-bit subclients column.  Stream-ordered. */
int dm_publish_totals(dm_ctx* ctx, void* dev_dst);

/* The publish fused into the tick: with a ring of n >= 3 device buffers (each 1 + R
 * records), the k-th writeback tick from this call on also writes what
 * dm_publish_totals would into bufs[k % n] -- each resource's record as the tick stores
 * its running sums, the validation flags OR-ed into record 0 -- and clears record 0 of
 * bufs[(k + 1) % n] for the next tick.  Three buffers keep a tick's block intact while
 * the pipelined exchange of the tick before (dm_hier_pipeline) still reads it.
 * A store whose one workgroup bin runs in two stream parts (dm_plan_info slot 17) keeps
 * one 32-bit flags word per part in record 0's first 8 bytes (part 0 the low word,
 * part 1 the high word): the request's flags are their OR, and the int64 read of those
 * bytes is nonzero exactly when the flags are.  This call clears record 0 of every
 * buffer (stream-ordered).  n = 0 turns it off. */
int dm_publish_ring(dm_ctx* ctx, int n, void* const* dev_bufs);

/* Layout of the exchange, set once on the root context (default: replicated, with
 * n_servers from each dm_hier_root_tick and stride 1 + R):
 *   shard_lo == NULL  replicated: every server holds all R resources of the root; the
 *                     root store holds R x n_servers rows (resource r: rows r*G .. r*G+G-1).
 *   shard_lo != NULL  sharded by resource id: n_servers + 1 non-decreasing
 *                     bounds from 0 to R; server g holds resources [shard_lo[g],
 *                     shard_lo[g+1]) and only it requests them; the root store holds one
 *                     row per resource (its owner's).
 * stride: records per server block in the gathered buffer (server g's dm_publish_totals
 * block starts at record g * stride), >= 1 + the largest shard; 0 = exactly that. */
int dm_hier_layout(dm_ctx* root, int n_servers, const int64_t* shard_lo, int64_t stride);

/* One exchange round of the intermediate-server hierarchy, on the root store of this
 * server's device (every server evaluates the root redundantly):
 *
 *   performRequests        go/server/doorman/server.go:227-323  -> the gathered dm_publish_totals blocks
 *   GetServerCapacity      go/server/doorman/server.go:822-901  -> the root's round below
 *   Server.LoadConfig      go/server/doorman/server.go:187-218  -> this server's new leaf templates
 *   Resource.LoadConfig    go/server/doorman/resource.go:117-125
 *
 * dev_gathered holds every server's dm_publish_totals block (dm_hier_layout).
 *   - Server g requests resource r when its SumWants > 0 (server.go:241): has 0
 *     (Has is never filled, :244/:873), wants = SumWants, subclients = Count.
 *     A server whose block carries validation flags requests nothing this round and
 *     its leaf keeps its templates (:268-272); see dm_hier_status.
 *   - The round's requests are decided one after another in server order, as the
 *     root's res.mu serialises GetServerCapacity calls (resource.go:103-104): Clean,
 *     then Learn or the resource's algorithm with the request's own values against
 *     the store as the earlier requests' Assigns left it, then its Assign
 *     (store.go:153-167) -- so the grants never exceed what the reference gives.
 *     Servers that do not request keep their root lease until it expires.
 *   - The leaf (`leaf`: this server's store of its own resources, same device) gets
 *     its new templates: a requested resource takes the grant as capacity, the grant's
 *     expiry in Unix seconds as parent expiry, and the root's algorithm (kind, lease
 *     length, refresh interval) and configured safe capacity (0 when unset,
 *     :293-296,:894); every other resource drops to the "*" default template
 *     (capacity 0, safe capacity 0, FAIR_SHARE, lease 20 s, refresh 1 s, no parent
 *     expiry; server.go:53-63,:305).  Learning-mode end times are kept (fixed when a
 *     resource is created, resource.go:153-163).  Without dm_hier_pipeline they are
 *     written in place, ordered before the leaf's next tick; with it they are staged.
 * 1 <= n_servers <= 64.  One stream-ordered launch; returns without waiting. */
int dm_hier_root_tick(dm_ctx* root, const void* dev_gathered, int n_servers, int64_t now_ns, dm_ctx* leaf,
                      int server);

/* Pipelined templates on a leaf (on = 1): each dm_hier_root_tick for this leaf stages
 * its templates instead of writing them, and every dm_apportion of the leaf first takes
 * the templates of the exchanges enqueued before the previous dm_apportion call -- one
 * tick of lag, as the reference's intermediate refreshes upstream on its own loop
 * (server.go:227-323) while it keeps serving clients -- so the exchange (publish,
 * all-gather, root round) can run on a stream of its own beside the next leaf tick.
 * on = 2 or 3: one or two ticks more (an exchange on its own stream then has a whole
 * tick to finish before the leaf needs it: the leaf never waits for it).  Off (0,
 * default) takes the newest staged templates. */
int dm_hier_pipeline(dm_ctx* leaf, int on);

/* Per-server outcome of the last dm_hier_root_tick (waits for it): status[g] = 0 when
 * server g's request was accepted, else DM_HIER_INVALID (a band with num_clients < 1,
 * server.go:863-866) and/or DM_HIER_COUNT_RANGE.  Returns the number of rejected
 * servers (>= 0) or a DM_E_* code. */
#define DM_HIER_INVALID 1u
#define DM_HIER_COUNT_RANGE 2u
int dm_hier_status(dm_ctx* root, uint32_t* status, int n_servers);

/* ---- one intermediate server's whole step in one call ----
 * The reference's intermediate serves its clients and refreshes its own lease upstream
 * on a loop of its own (server.go:227-323).  dm_hier_step does both for one step with no
 * host round trip in between: the leaf's writeback tick (dm_apportion, its block
 * published into the ring), then on the exchange stream the block gathered from every
 * server and the root's round (dm_hier_root_tick) staging this server's templates for the
 * leaf's next-but-one tick (dm_hier_pipeline).  The blocks are gathered by
 *   - the RCCL communicator of dm_hier_comm_init: one ncclAllGather over xGMI of every
 *     server's block (stride records each) into the gathered buffer;
 *   - without one, with one server: nothing (the root reads the ring block in place);
 *   - without one, with several servers (a rehearsal of one rank of a node on one GPU):
 *     this server's block copied into its slot, the other slots as the caller left them.
 * dm_hier_attach binds the pair once: the ring (nring >= 3 device blocks of `stride`
 * double2 records, as dm_publish_ring), the gathered buffer (n_servers x stride records;
 * unused with one server), the exchange stream (NULL: the leaf's), the server index; it
 * needs dm_hier_layout on the root and turns dm_hier_pipeline on for the leaf.  The
 * per-step host work is then a handful of stream operations: a step of a small shard
 * stays device-bound instead of host-bound. */
int dm_hier_attach(dm_ctx* leaf, dm_ctx* root, int server, void* const* ring, int nring, void* gathered,
                   void* exchange_stream);
int dm_hier_step(dm_ctx* leaf, dm_ctx* root, int64_t now_ns);
/* RCCL communicator of the exchange (librccl, loaded when first needed): rank 0 creates
 * the id (id_out: DM_RCCL_ID_BYTES bytes), every rank passes it to dm_hier_comm_init with
 * the node's rank count and its rank (collective: every rank must call it).  One rank
 * per GPU; the root context keeps the communicator until dm_destroy. */
#define DM_RCCL_ID_BYTES 128
int dm_rccl_unique_id(void* id_out);
int dm_hier_comm_init(dm_ctx* root, const void* id, int nranks, int rank);
/* What the exchange's communicator itself reports (ncclCommCount, ncclCommUserRank):
 * the ranks RCCL saw and this one's rank, so a multi-GPU run can show that RCCL, not
 * only torch.distributed, spans the node.  DM_E_STATE without a communicator. */
int dm_hier_comm_info(dm_ctx* root, int* nranks, int* rank);

/* Large resources (more than 4096 rows) run on 2048-row chunks in stream-ordered
 * launches (Clean + speculative round 1, round 1 again only where Clean released
 * subclients, FairShare round 2, the map, whose last-arriving chunk per resource writes
 * the record); every chunk re-derives the resource's totals (algorithm.go:156-204,
 * 259-279) from the previous launch's per-chunk partials with one fixed tree.  (The
 * one-launch and persistent-queue forms of rounds 2-3 lost to it and were retired in
 * round 4: DESIGN.md §4.3.) */

/* ---- profiling ---- */
int dm_set_profiling(dm_ctx* ctx, int on);
/* fills up to max entries; returns the number of kernel classes (>= 0) */
int dm_kernel_times(dm_ctx* ctx, dm_kernel_time* out, int max);
/* the names dm_kernel_times reports, in its order (static strings; no context or GPU
 * needed); returns the number of classes */
int dm_kernel_class_names(const char** names, int max);
int dm_reset_kernel_times(dm_ctx* ctx);
/* plan summary of the loaded store: small-resource tiles, items per dispatch bin (sub16x4,
 * sub32x4, wave64x4, block128x4, block128x8, block256x8, the 2049-4096-row bin,
 * sub8x2, sub16x2), large resources, large chunks, leases, then the bins' shapes (bit 0:
 * the 2049-4096-row bin runs on 512 x 8 workgroups, else 256 x 16; bit 1: the
 * 513-1024-row bin on one wave per resource, 64 x 16, else 128 x 8), 3/4 of the redo's
 * full-build workgroups the GPU holds at once (its grid bound), and 1 (every store may
 * speculate: the redo by teams needs only 64 co-resident workgroups), and 1 when the
 * work classes' auxiliary streams each have a hardware queue of their own, and the
 * stream parts of the store's one workgroup bin (2: its halves run on two auxiliary
 * streams, unjoined from tick to tick; else 1), and the queue assignment the context chose
 * for its class streams (perm[0] + 4 perm[1] + 16 perm[2] + 64 perm[3]: class stream i
 * runs on the i-th auxiliary queue's perm[i]-th creation; timed on the context's first
 * forked writeback ticks, -1 until then); returns 19 */
int dm_plan_info(dm_ctx* ctx, int64_t* out, int max);
/* row-state summary of the device store (synchronous): dense resources (every row a
 * live follower with one subclient count: a tick reads 24 B per lease, not 28),
 * their rows, resources that may hold explicit expiries, resources; returns 4 */
int dm_store_stats(dm_ctx* ctx, int64_t* out, int max);

/* ---- round-oriented GetCapacity dispatch (dm_server.cpp) ----
 *
 * The request path of the reference server over a device-resident store:
 *
 *   Server.GetCapacity      go/server/doorman/server.go:730-796  -> dm_server_get_capacity + dm_server_tick
 *   Server.getCapacity      go/server/doorman/server.go:798-817  -> dm_server_tick (one batch per round)
 *   Server.ReleaseCapacity  go/server/doorman/server.go:668-714  -> dm_server_release_capacity
 *   Resource.Decide         go/server/doorman/resource.go:100-113 -> Clean + Learn/Algorithm in the tick
 *   LeaseStore (client-id)  go/server/doorman/store.go:68-167     -> client -> row map over the columnar store
 *   SetSafeCapacity         go/server/doorman/resource.go:81-96   -> dm_server_lease(.safe_capacity)
 *
 * Requests queued during a round are decided together by dm_server_tick: the
 * store first drops expired leases (Clean, store.go:169-181) and released
 * clients (store.go:142-151); then every request is decided by Resource.Decide in
 * queue order, each seeing the Assigns (store.go:153-167) of the requests before it
 * on its resource (dm_decide: the request's own has, wants and subclients for its
 * client, new clients absent from the store until their first Assign).  A round is
 * the reference's GetCapacity calls served one after another in queue order.  Clients that did not ask keep their
 * leases, which expire unless refreshed.  A round that fails leaves no leases
 * (dm_server_lease then reports an error for its tickets) and forgets the new
 * clients it had placed.  Resources are configured up front (the outcome of
 * the reference's LoadConfig; config parsing and glob matching stay there);
 * every resource's segment of the table grows when it runs out of free rows. */
typedef struct dm_server dm_server;

/* resource_ids: R NUL-terminated ids; cfg: their configuration (dm_config_load);
 * slots: initial rows per resource (grown on demand) */
int dm_server_create(int device, int64_t n_resources, const char* const* resource_ids, const dm_resource_cfg* cfg,
                     int64_t slots, dm_server** out);
void dm_server_destroy(dm_server* srv);
const char* dm_server_last_error(dm_server* srv);
/* queue one ResourceRequest of a GetCapacity (subclients = 1 there, >= 1 for a
 * server band, server.go:863-866: DM_E_ARGUMENT otherwise); *ticket indexes the
 * next dm_server_tick's leases; an unknown resource is DM_E_RANGE */
int dm_server_get_capacity(dm_server* srv, const char* client, const char* resource, double has, double wants,
                           int64_t subclients, int64_t* ticket);
/* queue a ReleaseCapacity of one client's lease on one resource */
int dm_server_release_capacity(dm_server* srv, const char* client, const char* resource);
/* decide every queued request at time now_ns (one batch) */
int dm_server_tick(dm_server* srv, int64_t now_ns);
/* the lease of a ticket of the last tick, as GetCapacity returns it
 * (server.go:783-796): capacity, expiry_time (unix s), refresh_interval (s),
 * and the resource's safe capacity (resource.go:81-96) */
int dm_server_lease(dm_server* srv, int64_t ticket, double* capacity, int64_t* expiry_time_s,
                    int64_t* refresh_interval_s, double* safe_capacity);
/* store state: number of clients holding a lease on a resource, and its running sums */
int dm_server_resource(dm_server* srv, const char* resource, int64_t* clients, int64_t* count, double* sum_has,
                       double* sum_wants);
/* the underlying context (profiling, dm_read_*) */
dm_ctx* dm_server_ctx(dm_server* srv);

#ifdef __cplusplus
}
#endif
#endif
