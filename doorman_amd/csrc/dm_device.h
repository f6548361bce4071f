// dm_device.h — structures shared by the host runtime and the gfx950 kernels.
#pragma once
#include <stdint.h>

namespace dm {

constexpr int64_t kReleased = INT64_MIN;
constexpr int64_t kNs = 1000000000LL;

// The subclients column (4 B per lease) also says where a lease's expiry lives:
//   bit 31 clear         a follower: subclients = the value; its expiry is its
//                        resource's follow_exp (every lease a writeback tick grants on
//                        one resource expires at now + lease length, store.go:161),
//                        so the tick neither reads nor writes an 8-B expiry per lease
//   kSubReleased         released by Clean / Release: subclients 0, expiry DM_RELEASED
//   bit 31 set otherwise explicit: subclients = value & 0x7FFFFFFF, expiry in the
//                        expiry column (rows loaded or upserted by the host)
// A writeback tick leaves every row a follower or released; the values a lease
// reads back (dm_read_store / dm_read_leases) are the same either way.
constexpr uint32_t kSubExplicit = 0x80000000u;
constexpr uint32_t kSubReleased = 0xFFFFFFFFu;
constexpr int64_t kSubMax = 0x7FFFFFFE;  // largest subclients value a row holds

// Dispatch bins.  A segment of n rows goes to:
//   n <= kSmallMax            : tiles of consecutive resources, one resource per thread (k_tile_small)
//   n <= 16 / 32              : 2- to 8-lane groups, 3-4 rows per lane (bins 7, 8; SubBins below)
//   n <= 64 / 128             : 16- / 32-lane groups, 4 rows per lane, 4 / 2 resources per wave (bins 0, 1)
//   n <= 256                  : one wave per resource, 4 rows per lane (4 resources per workgroup)
//   n <= 512 / 1024           : one 128-thread workgroup, 4 / 8 rows per thread in VGPRs (bins 3, 4)
//   n <= 2048                 : one 256-thread workgroup, 8 rows per thread (bin 5)
//   n <= 4096                 : one 256 x 16 or 512 x 8 workgroup (bin 6, kBin6Wide below)
//   n >  kLargeMin            : multi-workgroup chunks of kChunkRows rows
constexpr int kSmallMax = 4;  // (8: 5-8 rows in the tiles, 2.9 TB/s at 8 rows, one resource per thread; 16 and 32 lost +8 / +25 us on C2)
static_assert(kSmallMax <= 32, "k_tile_small keeps a resource's live rows in a 32-bit mask");
constexpr int kLargeMin = 4096;
constexpr int kChunkRows = 2048;
constexpr int kNumBins = 9;  // sub16x4, sub32x4, wave64x4, block128x{4,8}, block256x8, the 2049-4096 bin, sub8x2, sub16x2
// Bin 6 (2049-4096 rows) runs on 256 x 16 workgroups (4 wave slots each: they find room
// beside the other classes' workgroups; C2's bin under contention 63.6 -> 55.0 us of
// event time) or, when it holds most of the store's rows, on 512 x 8 (12.7 against
// 15.2 us alone): launch_bin* take kBin6Wide for the latter.
constexpr int kBin6Wide = 9;
// Bin 4 (513-1024 rows) on one wave per resource (64 lanes x 16 rows: every reduction a
// wave reduction, no LDS round or barrier) when most of its resources are FairShare,
// whose round 2 is one more reduction than ProportionalShare's (C1 FairShare 41.0-41.8
// -> 38.1-38.7 us; ProportionalShare 37.7-38.0 -> 39.0: profiles/r05_ab/b4_one_wave.txt).
constexpr int kBin4Wave = 10;
// Lease-table footprint (48 B per lease) above which a tick is taken to stream
// from HBM rather than partly from the 256 MiB Infinity Cache (launch_bin).
constexpr int64_t kStreamBytes = 1LL << 30;


// A tile of consecutive small resources (n <= kSmallMax) for k_tile_small: at most
// kTileRes resources and kTileRows rows, one 256-thread workgroup each.  Its rows are
// staged in LDS by the whole workgroup (coalesced), each resource's record is loaded by
// the thread that decides it (consecutive records: coalesced too), so a tile needs one
// memory round trip before its compute instead of the packed kernel's two.
constexpr int kTileRows = 1024;  // (512-row tiles: C2 +1.7 us)
constexpr int kTileRes = 256;
// A run of fewer than kTileMinRun consecutive small resources (a store whose small and
// larger resources interleave, as resource ids are handed out in no particular order)
// does not get a tile of its own (a workgroup for a handful of resources: a random mix
// of 2-6-row resources ran 314 us against 15 + 10 for its two classes alone,
// tools/overlap_probe.py): its resources go to list tiles, which name up to kTileRes
// scattered small resources (TileEntry) and stage each one's rows by its own thread.
constexpr int kTileMinRun = 64;
struct Tile {
  int32_t first_seg;  // list tile: its first entry in the tile list
  int32_t nseg;    // <= kTileRes
  int64_t row0;    // list tile: unused
  int32_t nrows;   // <= kTileRows
  int32_t list;    // 1: a list tile
};
struct TileEntry {
  int32_t seg;
  int32_t lds;  // the resource's first row in the tile's LDS rows
};

struct WorkItem {  // one resource of a size bin: no dependent load before its rows
  int32_t seg;
  int32_t n;   // rows (<= 4096) in bits 0-15; bits 16-23: the dense hint written by
               // writeback ticks (s0 > 0 when expl[seg] == s0 + 1, below), else 0;
               // bit 24: the resource also holds released rows (DevParams::rmask)
  int64_t lo;
};

// The sub-wave bins of one tick for k_subs, in launch order, each bin in several
// shapes G x R (G lanes per resource, R rows per lane; a bin's items ordered by shape,
// build_plan): bin 7 (5-16 rows) 2x3 (5-6), 2x4 (7-8), 4x3 (9-12), 4x4 (13-16); bin 8 (17-32) 8x3 /
// 8x4; bin 0 (33-64) 16x3 / 16x4; bin 1 (65-128) 32x3 / 32x4; bin 2 (129-256) 64x3 / 64x4.
// blocks[k] workgroups of 256 threads each (256 / G resources per workgroup).
// Power-of-two shapes alone leave a Zipf population's lanes mostly idle: its resources
// crowd at the low edge of every bin (a 9-row resource in 16 slots), and a sub-wave tick
// is bound by rows in flight, padded slots included; more rows per lane also beat wider
// groups at equal slots (tools/size_sweep.py, profiles/r06_size_sweep.md).
constexpr int kSubShapes = 12;
constexpr int kSubShapeG[kSubShapes] = {2, 2, 4, 4, 8, 8, 16, 16, 32, 32, 64, 64};
constexpr int kSubShapeR[kSubShapes] = {3, 4, 3, 4, 3, 4, 3, 4, 3, 4, 3, 4};
constexpr int kSubShapeBin[kSubShapes] = {7, 7, 7, 7, 8, 8, 0, 0, 1, 1, 2, 2};
struct SubBins {
  WorkItem* items[kSubShapes];
  int32_t n[kSubShapes];
  int32_t blocks[kSubShapes];
};

struct Chunk {  // kChunkRows rows of one large resource
  int32_t seg;
  int32_t lseg;  // index into the large-resource table
  int64_t row0;
  int32_t nrows;
  int32_t pad;
};

struct LargeSeg {
  int32_t seg;
  int32_t chunk_begin;
  int32_t chunk_end;
  int32_t pad;
};

// Per-chunk partial results of the large path (one slot per chunk).
struct Partials {
  // pass A: expired-row sums, all-row sums (recompute mode), uniformity flags
  int64_t* a_cnt;
  double* a_has;
  double* a_wants;
  int64_t* a_cnt_all;
  double* a_has_all;
  double* a_wants_all;
  int64_t* a_smin;
  int64_t* a_smax;
  int32_t* a_nan;
  // pass B: FairShare E / W, ProportionalShare extraCapacity / extraNeed
  double* b_x;
  double* b_y;
  int64_t* b_w;
  // pass C: FairShare extraExtra / wantExtraExtra at the common threshold T
  double* c_ee;
  int64_t* c_sgt;
  // map pass: sum of (gets - has) over live rows
  double* d_delta;
  // pass A: per thread of each chunk, bit k (row k*256+tid) of byte 0 = live, byte 1 =
  // explicit expiry, byte 2 = already marked released; passes B, C and the map read
  // wants (+ subclients for ProportionalShare) and not expiry
  uint32_t* live;
  // per large resource (kSegTotBytes each): pass A totals left by pass B's first
  // chunk, pass B totals left by pass C's first chunk, so the map reduces at most
  // one set of partials
  uint8_t* tot;
  // heterogeneous-subclient FairShare on the chain (only when the store may hold
  // such resources; nullptr otherwise -- they then go to the one-workgroup k_general):
  // per large resource the set of distinct subclient counts of its live rows (pass A
  // inserts, k_large_t reads and empties it), a HetRes record, per chunk the round-2
  // bucket partials (pass C)
  uint32_t* s_set;  // [large resources * 2 * kHetMaxS] open addressing, all ones = empty
  int32_t* s_n;     // [large resources] distinct counts inserted (> kHetMaxS: overflow)
  uint8_t* het;     // [large resources * sizeof(HetRes)]
  double* bk_w;     // [nchunks * kHetBuckets]
  int64_t* bk_s;
  int32_t* bk_c;
  // 1: pass B runs one workgroup per large resource (the store holds no
  // explicit-expiry rows, so pass A's speculative round 1 is exact)
  int32_t b_first;
  // 1: the last call that changed the store was a writeback tick through this chain
  // (uni and `live` are that tick's), so pass A reads no subclients column for chunks
  // with uni >= 0: a row live then holds uni, every other row is marked released
  int32_t s_live;
  // per chunk: the map leaves the resource's subclients count when every row it left
  // live holds that count, -1 otherwise
  int32_t* uni;
};
constexpr int kSegTotBytes = 128;

// The speculative chain (k_large_spec / k_large_redo, dm_kernels.hip): per large
// resource, the round-1 / round-2 totals and the live rows' count its last tick
// verified (or redid), used as this tick's speculation; the redo's inputs and meeting
// points.  Reductions over a resource's chunk partials here all take one fixed tree
// (wave 0, 64 lanes striding the chunks in order), so a total recomputed from the
// same partials is bit-identical to the stored one.
struct SpecTot {
  double bx, by;        // AggB of the last verified tick (FairShare E / W, ProportionalShare x / y)
  long long bi;
  double cee;           // AggC
  long long csgt;
  int32_t s0;           // the live rows' one subclient count
  int32_t valid;        // bx .. s0 hold a tick's totals
  uint32_t redo;        // this tick's speculation failed (set by k_large_spec, cleared by the redo)
  uint32_t arrive[3];   // arrival counters (reset by their last arriver)
  uint64_t ready[2];    // the redo's ready flags: its launch number + 1 once a total is stored
  // k_large_spec's verifier leaves the resource's actual pass-A totals and round 1
  // (equalShare from the running Count) for the redo
  long long a_cnt;
  double a_h, a_w;
  int32_t a_smin, a_smax, a_nan, pad;
  double abx, aby;
  long long abi;
};
struct SpecArgs {
  SpecTot* tot;     // [large resources]
  uint64_t seq;     // the redo's launch number
  int32_t* err;     // host-mapped: a redo chunk gave up waiting for its resource's others
  uint32_t* ring;   // [4]: per tick parity, "some resource marked" and the redo's chunk tickets
  int par;          // this tick's parity (the redo clears the other slots for the next tick)
  int nchunks;
  uint32_t* seen;   // host-mapped: whether the last redo launch found a resource marked
  const int32_t* team;  // k_large_redo_team: per team slot, (large resource) << 8 | member
  int nslots;           // team slots: min(chunks, kTeamMax) per large resource
};
constexpr int kTeamMax = 64;  // workgroups that redo one large resource together
constexpr int kHetMaxS = 256;                    // distinct subclient counts per resource on the chain
constexpr int kHetBuckets = 2 * kHetMaxS + 1;    // strictly between / equal to the sorted thresholds
struct HetRes {
  int32_t mode;  // 0: not heterogeneous FairShare; 1: decided on the chain; 2: handed to k_general
  int32_t K;     // distinct thresholds
  double T[kHetMaxS];       // ascending
  double bw[kHetBuckets];   // per bucket over the resource's chunks (k_large_e): sum of wants,
  int64_t bs[kHetBuckets];  // sum of subclients,
  int64_t bc[kHetBuckets];  // count of the wantExtra clients
};


// row -> resource lookup for store updates: seg_off plus, for every block of
// 2^kRowBlkShift rows, the resource holding its first row
constexpr int kRowBlkShift = 12;
struct RowIndex {
  const int64_t* seg_off;
  const int32_t* blk_seg;  // (N >> kRowBlkShift) + 2 entries
  int64_t R;
};

// store-update validation flags (k_check_rows)
constexpr uint32_t kUpdRange = 1u;   // row outside [0, N)
constexpr uint32_t kUpdDup = 2u;     // row twice in one call
constexpr uint32_t kUpdSub = 4u;     // subclients outside [0, kSubMax]
constexpr uint32_t kUpdNaN = 8u;     // NaN wants (FairShare then needs k_general)
constexpr uint32_t kUpdNotOne = 16u; // subclients != 1 (may make a resource heterogeneous)
constexpr uint32_t kUpdCount = 32u;  // packed values != set bits of the row mask
constexpr uint32_t kUpdReject = kUpdRange | kUpdDup | kUpdSub | kUpdCount;

// Per-resource configuration, AoS (one scalar burst per resource).
struct ResCfg {  // what every tick reads: 32 B
  double capacity;          // ResourceTemplate.capacity
  int64_t learning_end_ns;  // learningModeEndTime
  int64_t parent_expiry_ns; // Resource.expiryTime (INT64_MAX = nil)
  int32_t lease_len_s;      // Algorithm.lease_length (seconds, < 2^31, checked at load)
  int32_t kind;             // pb.Algorithm.Kind
};
struct ResCold {  // what only the readers and the hierarchy touch: 16 B
  double safe_capacity;     // NaN = unset (resource.go:91)
  int32_t refresh_s;        // Algorithm.refresh_interval (seconds; < 2^31, checked at load)
  int32_t pad;
};

// The store's running sums (store.go:105-111) and the expiry of the resource's
// follower rows (SetSafeCapacity's value is derived from count at read time).
// Whether any row of the resource may carry an explicit expiry is a separate byte
// per resource (DevParams::expl), written only when it changes.
struct ResAgg {  // 32 B, read and written by every tick
  int64_t count;
  double sum_has;
  double sum_wants;
  int64_t follow_exp;
};

struct DevParams {
  const int64_t* seg_off;
  // lease table (SoA).  out_* alias these in writeback mode, so no __restrict__.
  const double* wants;
  const double* has;
  const int32_t* sub;   // subclients in [0, kSubMax] + the expiry encoding above: 4 B per lease
  const int64_t* expiry;
  const ResCfg* cfg;
  const ResAgg* agg;  // running sums read by the tick (parity mode)
  // lease outputs
  double* out_gets;
  int64_t* out_expiry;
  double* out_wants;  // writeback only: released rows zeroed (else nullptr)
  int32_t* out_sub;   // writeback only
  ResAgg* res;        // per-resource results (== agg in writeback mode)
  uint8_t* expl;      // [R] per-resource row state: 1: some row may carry an explicit
                      // expiry (loaded, upserted, hierarchy-written); 0: every row follows
                      // its resource or is released; s0 + 1 in [2, 255] ("dense"): every
                      // row is a live follower with subclients == s0, so a tick need not
                      // read the subclients column (set by writeback ticks of the
                      // 128-thread group kernels, 257-1024 rows; upserts set 1, releases
                      // reset it to 0)
  // Released-row masks of the dense resources of the workgroup bins (257-4096 rows):
  // the resource starting at row lo owns the bytes from rel_mask_offset(lo), one
  // RelMask<R> entry per lane (bit k: row k*G + lane is released).  N/2 + 64 bytes.
  uint8_t* rmask;
  int64_t now;
  int32_t recompute;
  int32_t writeback;  // rows become followers / released in the store; out_expiry unused
  // dm_publish_ring: a writeback tick also writes what dm_publish_totals would (record
  // 1 + r = {SumWants, Count} as each resource's sums are stored, the validation flags
  // OR-ed into record 0) and clears its flags word in record 0 of the ring's next
  // buffer; nullptr: off.  A bin split into stream parts (dm_runtime.cpp) runs its parts
  // unjoined from tick to tick, so each part owns a 32-bit flags word of record 0
  // (pub_word: 0 or 1; the first 8 bytes read as one int64 hold their OR in either
  // half) and clears only that word, from its first resource (pub_first), in the next
  // buffer; pub_word -1: the tick's only launch that publishes the first resource
  // (word 0, and it clears the whole record).
  double2* pub;
  double2* pub_clear;
  int32_t pub_word;
  int32_t pub_first;
};

// The validation flags of a published block's record 0: the OR of its two flags words
// (DevParams::pub_word).
__host__ __device__ inline uint32_t pub_flags(double x) {
  long long b;
  __builtin_memcpy(&b, &x, 8);
  return (uint32_t)b | (uint32_t)((unsigned long long)b >> 32);
}

// dm_decide: one resource and its requests [qlo, qhi) in the caller's order; the
// resource's rows are copied to scratch rows [scr, scr + n) that take each
// decision's Assign before the next request is decided
template <int R> struct RelMask { using T = uint8_t; };   // R <= 8 rows per lane
template <> struct RelMask<16> { using T = uint16_t; };
// 4-aligned, lo/2 - 4 < offset <= lo/2: a resource of n rows owns at least
// 4 * floor(n / 8) bytes before the next one's, enough for G entries of R/8 bytes
// in every workgroup bin (n > G * R / 2, R >= 4)
constexpr int64_t rel_mask_offset(int64_t lo) { return (lo >> 3) << 2; }

// A dense resource stays dense through store updates (round 6, configs[4]'s rounds):
// a release marks its row in the released-row mask (rmask) and the work item's hint
// (bit 24, "has released rows") instead of ending the dense state, and an arrival onto
// one of its rows -- the resource's subclient count, the expiry Assign gives (now +
// lease length) at or after the followers' -- clears the row's released bit and sets
// it in the arrival mask (amask) and the item's bit 25 instead of marking the resource
// explicit.  The tick then reads neither the subclients nor the expiry column for it:
// arrival rows are live followers unless the followers themselves have lapsed, when
// the resource takes the column path (the arrivals' own expiries decide); a writeback
// tick turns the arrivals into followers and clears the arrival mask.
// Both masks live in the resource's rmask bytes (rel_mask_offset): lane t's entry of
// R bits (bit k: row k * G + t), RelMask<R> wide; the arrival entry shares the byte
// (high nibble) for R <= 4, else follows the G released-row entries.
struct MaskPos {
  int32_t roff, rbit;  // released-row mask: byte offset from the resource's first mask byte, bit
  int32_t aoff, abit;  // arrival mask
};
__host__ __device__ inline MaskPos mask_pos(int G, int R, int i) {
  const int t = i % G, k = i / G, es = R <= 8 ? 1 : 2;
  MaskPos m;
  m.roff = t * es + (k >> 3);
  m.rbit = k & 7;
  if (R <= 4) {
    m.aoff = m.roff;
    m.abit = m.rbit + 4;
  } else {
    m.aoff = G * es + t * es + (k >> 3);
    m.abit = k & 7;
  }
  return m;
}
// What the update kernels need for it: the resource's work item (bins 3-6) and the
// bins' shapes (G x R: bin 3 128 x 4, bin 4 128 x 8 or 64 x 16, bin 5 256 x 8, bin 6
// 256 x 16 or 512 x 8).
struct DenseUpd {
  const int32_t* item_of;  // [R]: bin << 24 | the item's index in its bin, -1 outside bins 3-6
  WorkItem* bins[4];
  int32_t bin4_wave, bin6_wide;
  uint8_t* rmask;
};
__host__ __device__ inline void bin_shape(int bin, int bin4_wave, int bin6_wide, int* G, int* R) {
  *G = bin == 3 ? 128 : bin == 4 ? (bin4_wave ? 64 : 128) : bin == 5 ? 256 : (bin6_wide ? 512 : 256);
  *R = bin == 3 ? 4 : bin == 4 ? (bin4_wave ? 16 : 8) : bin == 5 ? 8 : (bin6_wide ? 8 : 16);
}

struct ReqItem {
  int32_t seg;
  int32_t fast;  // 1 + its slot of the fast path (FastItem), 0: decided by k_decide only
  int64_t qlo, qhi;
  int64_t scr;
};
struct ReqArgs {
  const int64_t* rows;  // the row the request's lease is written to (its client's row, or a free row)
  const double* has;    // Request.Has (read by Learn only)
  const double* wants;
  const int64_t* sub;
  double* gets;
  int64_t* expiry;
  // the round's working copy of the requested resources' rows (store.Assign target)
  double* sc_has;
  double* sc_wants;
  int32_t* sc_sub;  // subclients of a live row, -1 for a row absent after Clean
  const struct FastRes* fast;  // the fast path's verdict per slot (k_decide skips items it decided)
};

// dm_decide's fast path (dm_decide_fast.hip) for a resource with many requests in a
// round whose requests keep every count (each requester a live row asking with the
// subclients every live row holds): equalShare is then constant through the round,
// FairShare round 1 / ProportionalShare's sums move by each Assign's own row only
// (prefix scans over the requests), FairShare round 2 at each request's threshold is
// a count / sum of the wants between deservedShare and T over the store as the earlier
// Assigns left it (sorted wants + sorted per-block Assign events), and only
// sumHas's recurrence (and ProportionalShare's sumWants test) stays sequential.
constexpr int kFdMin = 64;       // requests on one resource before the fast path is tried
constexpr int kFdBlock = 2048;   // requests per Assign-event block (2 events each)
constexpr int kFdRows = 4096;    // rows per workgroup of the fast path's row passes
constexpr double kFdMaxAbs = 1e300;  // |wants| and |capacity| bound: no overflow in the sums
constexpr int kFdChunk = 1024;   // scan elements per workgroup (4 per thread)
struct FastItem {
  int32_t item;  // index of the resource's ReqItem
  int32_t nblk;  // event blocks: ceil(K / kFdBlock)
  int64_t k0, K; // its requests [k0, k0 + K) of the round (grouped order)
  int64_t m0;    // offset of its sorted-wants area (n + 1 entries)
  int64_t e0;    // offset of its events (2 K)
  int64_t b0;    // first event block (global block index)
  int64_t n;     // rows of the resource
  int64_t c0;    // first row chunk (kFdRows rows each; global chunk index)
  int32_t nch;   // row chunks
  int32_t repeats;  // 1: some row is requested twice (the grants then need the sequential recurrence)
};
struct FdScan {  // one scanned element: double-double sums and an integer count
  double xh, xl;  // FairShare: extra (sum of d - w for w < d); ProportionalShare: extraCapacity
  double yh, yl;  // ProportionalShare: extraNeed
  double zh, zl;  // ProportionalShare: sumWants
  long long i;    // FairShare: wantExtra (subclients of rows with w > d)
};
struct FdClean {  // one row chunk's Clean partials
  long long cnt;  // subclients Clean releases
  double h, w;    // their has / wants
  int smin, smax; // live rows' subclients range
  int bad;        // some live row's wants NaN, infinite or beyond kFdMaxAbs
  int nlive;
};
struct FastRes {
  int32_t ok;    // 1: the fast path decides this resource's requests
  int32_t kind;
  int32_t s0;    // the one subclients count
  int32_t ok0;   // the rows qualify (before the requests are checked)
  int32_t bad;   // some request does not qualify (atomic OR)
  int32_t pad;
  double C, eq, d;
  long long count, nlive;
  double sum_has, sum_wants;  // after Clean
  FdScan init;                // the totals over the live rows before the round
  int64_t exp_out;
};
struct FdLind {  // the available-capacity recurrence a' = max(a + c, 0) composed: x -> max(x + A, B)
  double ah, al;
  double bh, bl;
};
struct FastArgs {
  const FastItem* fi;
  FastRes* fr;
  const int64_t* prev;  // [n requests] the previous request of the round on the same row, or -1
  double* pw;           // [n requests] the row's wants before the request
  double* v;            // [n requests] the request's grant before the avail cap (FS), or PS's round-1 grant
  FdScan* sc;           // [n requests] per-request deltas -> exclusive prefix (running totals)
  double* keys;         // [sum n + 1] live wants (+inf for absent rows) -> sorted into keys_s
  double* keys_s;
  FdScan* ps;           // [sum n + 1] exclusive prefix sums of the sorted wants
  double* ev_in;        // [sum 2K] Assign events: wants inserted (+1) / replaced (-1)
  int32_t* evs_in;
  double* ev;           // sorted within each block
  int32_t* evs;
  int32_t* ecnt;        // [blocks * (2 kFdBlock + 1)] exclusive prefix of the signs
  double2* esum;        // ... and of sign * wants (double-double)
  int32_t* bdc;         // [blocks] signed count / sum of the block's events <= d
  double2* bds;
  FdClean* pc;          // [row chunks] Clean partials
  FdScan* pt;           // [row chunks] totals partials
  FdLind* ld;           // [n requests] the recurrence's steps -> exclusive compositions
};

// dm_hier_root_tick: one exchange round of the hierarchy's root (k_hier_tick)
constexpr int kHierMaxServers = 64;     // one lane per server row, whole resources per wave
constexpr uint32_t kHierInvalid = 1u;    // a band with num_clients < 1: InvalidArgument (server.go:863-866)
constexpr uint32_t kHierCountRange = 2u; // Count > kSubMax: beyond the root's 32-bit subclients column
// A server's published block (dm_publish_totals): record 0 = {its request's
// validation flags as u64 bits, 0}, record 1 + i = {SumWants, Count as bits} of the
// i-th resource it holds; blocks sit `stride` records apart in the gathered buffer.
struct HierArgs {
  const double2* gathered;  // [G][stride]
  int64_t stride;
  const int64_t* shard_lo;  // [G + 1] sharded layout (server g holds resources [lo[g], lo[g+1])); nullptr: replicated
  uint32_t* status_out;     // [G] this round's flags, for dm_hier_status
  ResCfg* leaf_cfg;         // where this server's new templates go (its leaf's, or a staged slot)
  ResCold* leaf_cold;
  const ResCfg* leaf_prev_cfg;   // the templates a rejected round keeps (== leaf_cfg when written in place)
  const ResCold* leaf_prev_cold;
  const ResCold* root_cold; // the root's safe capacity / refresh interval
  int64_t R;
  int64_t leaf_lo;          // first resource of this server's leaf (0 when replicated)
  int64_t r_lo, r_hi;       // the resources this launch decides: this server's own range when
                            // sharded (no other server's leaf reads the rest), else [0, R)
  int G;                    // servers
  int K;                    // root rows per resource: G (replicated) or 1 (sharded: its owner's)
  int server;
  int pad;
};

}  // namespace dm
