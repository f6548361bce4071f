// dm_runtime.cpp — host runtime behind include/doorman_hip.h.
//
// Owns the device-resident columnar lease store (one context per GPU), builds
// the size-binned dispatch plan from the segment offsets, launches a tick on the
// context's HIP stream and reads results back.  See DESIGN.md §3-§5.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: librccl is loaded when the first communicator is made

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/doorman_hip.h"
#include "dm_device.h"

namespace dm {
hipError_t launch_tile_small(const DevParams& p, const Tile* tiles, const TileEntry* list, int n, hipStream_t st);
hipError_t launch_bin(int bin, const DevParams& p, WorkItem* segs, int n, int32_t* glist, int32_t* gcount,
                      hipStream_t st);
hipError_t launch_subs(const DevParams& p, const SubBins& sb, int32_t* glist, int32_t* gcount, hipStream_t st);
hipError_t launch_bin_dense(int bin, const DevParams& p, WorkItem* segs, int n, int32_t* queue, int32_t* qcnt, int par,
                            int32_t* glist, int32_t* gcount, int32_t* guard, hipEvent_t done, hipStream_t st);
int redo_blocks_per_cu();
hipError_t launch_large_spec(int phase, const DevParams& p, const Chunk* chunks, int nchunks, const LargeSeg* ls,
                             const Partials& P, const SpecArgs& S, int redo_grid, int32_t* glist, int32_t* gcount,
                             hipStream_t st);
hipError_t launch_count_undense(const WorkItem* items, int n, unsigned long long* rec, unsigned long long epoch,
                                hipStream_t st);
hipError_t launch_bin_rest(int bin, const DevParams& p, WorkItem* segs, int n, int32_t* queue, int32_t* qcnt, int par,
                           int32_t* host_count, int rest_grid, int32_t* glist, int32_t* gcount, hipEvent_t done,
                           hipStream_t st);
hipError_t launch_large(int phase, const DevParams& p, const Chunk* chunks, int nchunks, const LargeSeg* ls, int nls,
                        const Partials& P, int32_t* glist, int32_t* gcount, hipStream_t st);
hipError_t launch_general(const DevParams& p, const int32_t* glist, const int32_t* gcount, int blocks,
                          hipStream_t st);
hipError_t launch_upsert(int64_t n, const int64_t* rows, const double* has, const double* wants, const int64_t* sub,
                         const int32_t* sub32, const int64_t* expiry, const ResCfg* cfg, int64_t now,
                         const RowIndex& ix, double* s_has, double* s_wants, int32_t* s_sub, int64_t* s_exp,
                         ResAgg* agg, uint8_t* expl, const uint32_t* flags, const DenseUpd& du, hipStream_t st);
hipError_t launch_release(int64_t n, const int64_t* rows, const RowIndex& ix, double* s_has, double* s_wants,
                          int32_t* s_sub, int64_t* s_exp, ResAgg* agg, uint8_t* expl, const uint32_t* flags, const DenseUpd& du,
                          hipStream_t st);
hipError_t launch_check_rows(int64_t n, const int64_t* rows, int64_t N, uint32_t* bitmap, const double* wants,
                             const int64_t* sub, const int32_t* sub32, uint32_t* flags, hipStream_t st);
hipError_t launch_clear_rows(int64_t n, const int64_t* rows, int64_t N, uint32_t* bitmap, hipStream_t st);
hipError_t launch_resolve_rows(int64_t n, const int64_t* rows, int64_t off, const int32_t* sub, const int64_t* expiry,
                               const RowIndex& ix, const ResAgg* agg, int64_t* out_exp, int64_t* out_sub,
                               hipStream_t st);
hipError_t launch_gather_leases(int64_t n, const int64_t* rows, const double* gets, const int64_t* expiry,
                               double* out_gets, int64_t* out_exp, hipStream_t st);
hipError_t launch_publish(int64_t R, const ResAgg* agg, void* dst, uint32_t* sync, hipStream_t st);
hipError_t launch_update_wants(int64_t n, const int64_t* rows, const double* wants, const RowIndex& ix,
                               const int32_t* s_sub, double* s_wants, ResAgg* agg, const uint32_t* flags,
                               hipStream_t st);
hipError_t launch_update_wants_mask(int64_t nwords, const uint64_t* mask, int64_t first_row, int64_t N,
                                    int64_t n_values, const double* wants, int64_t* block_sums, int32_t* word_pre,
                                    const RowIndex& ix, const int32_t* s_sub, double* s_wants, ResAgg* agg,
                                    uint32_t* flags, hipStream_t st, int phase, int64_t vlo, int64_t vhi);
hipError_t launch_carry_reject(const uint32_t* from, uint32_t* to, hipStream_t st);
hipError_t launch_decide(const DevParams& p, const ReqItem* items, int nitems, const ReqArgs& q, hipStream_t st);
hipError_t fd_rows(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                   const FastArgs& fa, hipStream_t st);
hipError_t fd_item(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                   const FastArgs& fa, FdScan* part, hipStream_t st);
hipError_t fd_item_sorted(const DevParams& p, const ReqItem& it, const FastItem& fi, int slot, const ReqArgs& q,
                          const FastArgs& fa, FdScan* part, hipStream_t st);
hipError_t fd_sort_keys(void* temp, size_t* bytes, const double* in, double* out, int64_t n, hipStream_t st);
hipError_t fd_sort_pairs(void* temp, size_t* bytes, const double* kin, double* kout, const int32_t* vin,
                         int32_t* vout, int64_t n, int nseg, const int64_t* begin, const int64_t* end,
                         hipStream_t st);
hipError_t launch_hier_tick(const DevParams& p, const HierArgs& ha, hipStream_t st);
}  // namespace dm

using namespace dm;

namespace {

thread_local std::string g_last_error;

// kernel classes for profiling
enum KClass {
  KC_SMALL = 0,
  KC_BIN0,  // wave64 .. 256x16
  KC_LARGE_A = KC_BIN0 + kNumBins,
  KC_LARGE_B,
  KC_LARGE_C,
  KC_LARGE_MAP,
  KC_LARGE_FIN,
  KC_GENERAL,
  KC_UPSERT,
  KC_RELEASE,
  KC_SUBS,
  KC_DENSE3,  // the workgroup bins' split form (bins 3-6): dense kernel, then the rest kernel
  KC_DENSE4,
  KC_DENSE5,
  KC_DENSE6,
  KC_REST3,
  KC_REST4,
  KC_REST5,
  KC_REST6,
  KC_PUBLISH,   // dm_publish_totals
  KC_HIER_ROOT, // dm_hier_root_tick
  KC_LARGE_T,   // heterogeneous FairShare on the chain: thresholds,
  KC_LARGE_CH,  // bucket partials,
  KC_LARGE_E,   // bucket totals,
  KC_LARGE_MH,  // the map
  KC_DECIDE,    // dm_decide: the round's device work (fast path + k_decide)
  KC_LARGE_SPEC, // the speculative chain: k_large_spec,
  KC_LARGE_REDO, // k_large_redo
  KC_HIER_GATHER, // dm_hier_step's gather of the servers' blocks (ncclAllGather, or a rehearsal's copy)
  KC_COUNT
};
// bin 6 (2049-4096 rows) runs on 256 x 16 or 512 x 8 workgroups (kBin6Wide):
// "block2k4k" names the bin, dm_plan_info says which shape ran
const char* kClassNames[KC_COUNT] = {"small_tiles", "sub16x4",    "sub32x4",    "wave64x4",   "block128x4",
                                     "block128x8",   "block256x8", "block2k4k",  "sub8x2",    "sub16x2",
                                     "large_a",      "large_b",
                                     "large_c",      "large_map",  "large_fin",  "general",    "store_upsert",
                                     "store_release", "subs_merged", "block128x4_dense",
                                     "block128x8_dense", "block256x8_dense", "block2k4k_dense",
                                     "block128x4_rest", "block128x8_rest", "block256x8_rest", "block2k4k_rest",
                                     "hier_publish",
                                     "hier_root", "large_t", "large_c_het", "large_e", "large_map_het", "decide",
                                     "large_spec", "large_redo", "hier_gather"};

template <typename T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (count == 0) return hipSuccess;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e == hipSuccess) n = count;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct ProfEvent {
  int cls;
  hipEvent_t a, b;
};

}  // namespace

struct dm_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // auxiliary streams: independent size bins of one tick run concurrently
  static constexpr int kAux = 4;
  // auxiliary stream of each work class: bins 0..kNumBins-1, small tiles, large chain
  // (round 4 moved every bin to each other stream in A/Bs: this split won every one)
  // (round 5, with the small tiles: bin 3 on stream 3 112.8-117.3 us, on stream 1
  // 112.8-114.2, bin 6 on stream 3 127-129, against 111.0-112.4 us; profiles/r05_c2_classes.md)
  static constexpr int kClassStream[kNumBins + 2] = {2, 2, 2, 2, 1, 1, 1, 2, 2, 3, 0};  // C2: 200 -> 189 us (small class alone)
  // this store's assignment (plan_streams): kClassStream, except that on a store that
  // leaves some auxiliary stream without work, classes that would share a stream move
  // onto the idle ones (a shard of a Zipf population holds only some classes)
  int class_stream[kNumBins + 2] = {2, 2, 2, 2, 1, 1, 1, 2, 2, 3, 0};
  int64_t h_shape_lo[kSubShapes] = {}, h_shape_n[kSubShapes] = {};  // sub-wave shapes' items within their bins
  hipStream_t aux[kAux] = {};
  bool aux_own_queue = false;  // each auxiliary stream has a hardware queue of its own (CU mask)
  uint64_t aux_seq = 0;        // the stream set's creation order in the process (take_aux)
  hipStream_t cpy = nullptr;  // store-update column copies (overlap a running tick)
  hipEvent_t ev_stage[2] = {};  // staged update copies -> per-chunk validation
  // Cross-stream order between the context's streams (fork / join of a tick's work
  // classes, the pipelined hierarchy's template slots, dm_stream_wait): an event
  // recorded on the producing stream and waited on by the consuming one.  An event wait
  // idles the consuming queue ~12-20 us on the box (tools/xs_probe.py); stream-memory
  // tokens (hipStreamWriteValue64 / WaitValue64, which this ROCm runs as blit kernels
  // of 3-5 us each plus a dispatch gap) measured no cheaper per step (round 4: 75.0 vs
  // 72.2 us per N = 8 shard step) and were retired in round 5, as was the tick-done
  // word (the tick's last kernels' stop events replaced it: tick_ev below).  A wait on
  // a token signalled on the waiting stream itself is skipped (stream order).
  static constexpr int kTplSlots = 4;  // staged templates: in use + pending (lag 2) + the one being written
  enum : int {
    XS_FORK = 0,
    XS_JOIN0 = 1,                       // + aux stream
    XS_READY0 = XS_JOIN0 + kAux,        // + template slot: the root round wrote it
    XS_FREE0 = XS_READY0 + kTplSlots,   // + template slot: the ticks that read it are done
    XS_LEAF = XS_FREE0 + kTplSlots,     // leaf stream -> the root round's stream
    XS_ROOT,                            // root stream -> the leaf (unpipelined, separate streams)
    XS_EXT,                             // dm_stream_wait
    XS_N
  };
  struct XsTok {
    int w = 0;
    hipStream_t s = nullptr;  // the stream it was signalled on
    bool rec = false;         // recorded (else the wait records on s first: lazy signal)
  };
  // A pipelined leaf's staged templates from another stream: the host waits for the
  // exchange that made them and the leaf's stream gets no barrier (a queue waiting on
  // another queue here costs ~12-16 us even when the signal is long set -- the step of
  // an N = 8 shard idled that long every tick, tools/step_trace.py); the host stays at
  // most ~one step ahead, the device never waits.
  hipEvent_t xs_ev[XS_N] = {};
  hipError_t xs_signal(int w, hipStream_t s, XsTok* tok) {
    tok->w = w;
    tok->s = s;
    tok->rec = true;
    return hipEventRecord(xs_ev[w], s);
  }
  // A signal recorded only if a wait on another stream needs it, then at that wait:
  // it orders after everything the signalling stream holds by then (never less than
  // at signal time), and a same-stream consumer costs nothing.
  void xs_signal_lazy(int w, hipStream_t s, XsTok* tok) {
    tok->w = w;
    tok->s = s;
    tok->rec = false;
  }
  hipError_t xs_wait(const XsTok& tok, hipStream_t s) {
    if (tok.s == s || tok.s == nullptr) return hipSuccess;  // same stream, or known complete
    if (!tok.rec) return xs_order(tok.w, tok.s, s);
    return hipStreamWaitEvent(s, xs_ev[tok.w], 0);
  }
  hipError_t xs_order(int w, hipStream_t from, hipStream_t to) {
    if (from == to) return hipSuccess;
    XsTok t;
    hipError_t e = xs_signal(w, from, &t);
    return e == hipSuccess ? xs_wait(t, to) : e;
  }
  std::string err;

  int64_t R = 0, N = 0;
  bool store_loaded = false, cfg_loaded = false;
  // A device-side invariant failed (a redo workgroup gave up waiting, a dense kernel
  // queued an item on a tick that skipped its rest kernel: the host-mapped words
  // below).  The tick that tripped it may have written wrong leases and sums into the
  // store, so every call that reads, updates or ticks the store refuses it from then
  // on (DM_E_INTERNAL) until dm_store_load replaces it.
  bool store_lost = false;
  std::string lost_msg;
  // the store may hold explicit-expiry rows: set by every call that can write one
  // (load, upserts, decide, the root's tick), cleared by a writeback tick (which
  // turns every live explicit row into a follower).  Without them pass A's
  // speculative round 1 is exact and pass B runs one workgroup per large resource.
  bool expl_rows = true;
  // the last call that changed the store was a writeback tick through the chain
  // (Partials::s_live): cleared at the start of every tick and by every call that
  // writes a subclients word or releases a row
  bool chain_live_ok = false;
  // Row epoch: bumped by every call that writes rows (loads, plans, upserts, releases,
  // wants refreshes, decide, the root's tick) -- never by a tick.  Within one epoch a
  // writeback tick leaves every dense workgroup-bin resource dense (dm_kernels.hip),
  // so a bin verified all-dense once in the epoch (k_count_undense) can skip its
  // k_block_rest: nothing can be queued.
  uint64_t row_epoch = 1;
  void rows_changed() {
    chain_live_ok = false;
    row_epoch += 1;
  }
  std::vector<int64_t> h_seg_off;
  std::vector<int64_t> h_refresh_s;

  // lease table
  DBuf<int64_t> seg_off;
  DBuf<int32_t> blk_seg;  // RowIndex coarse index
  RowIndex row_index() const { return RowIndex{seg_off.p, blk_seg.p, R}; }
  DBuf<double> wants, has;
  DBuf<int32_t> sub;  // subclients, 4 B per lease on the device (the ABI carries int64)
  DBuf<int64_t> expiry;
  // running sums + the followers' expiry, AoS (32 B)
  DBuf<ResAgg> agg;
  DBuf<uint8_t> expl;  // per resource: rows may carry explicit expiries (DevParams::expl)
  DBuf<uint8_t> rmask;  // released-row masks of dense workgroup-bin resources (DevParams::rmask)
  DBuf<int32_t> item_of;  // [R]: bin << 24 | item index for bins 3-6, else -1 (DenseUpd)
  // config, AoS: what every tick reads (32 B), and the rest (safe capacity, refresh)
  DBuf<ResCfg> cfg;
  DBuf<ResCold> cold;
  // outputs of a non-writeback tick
  DBuf<double> out_gets;
  DBuf<int64_t> out_expiry;
  DBuf<ResAgg> res;
  bool last_writeback = false, have_result = false;
  // the workgroup bins' items carry dense hints: set by a writeback tick, kept by the
  // store updates (which keep a dense resource's state or end it: DenseUpd), cleared by
  // a new store
  bool hints_set = false;
  int64_t seg_uniform = 0;  // rows per resource when every resource has the same count, else 0
  // A forked tick's work classes run on the auxiliary streams.  Normally they are
  // joined back into the context stream at the end of the tick; with DM_DEFER_JOIN
  // the join waits for the next library call that needs it (each cross-queue hop
  // costs ~20 us on the GPU, so back-to-back ticks keep every class streaming).
  // aux_pending: class work not yet joined into the context stream.
  // main_dirty: the context stream holds work the auxiliary streams have not
  // waited for (the next fork must record an event).
  bool aux_pending = false, main_dirty = true;
  hipError_t join_aux() {
    if (!aux_pending) return hipSuccess;
    aux_pending = false;
    aux_unjoined = 0;
    for (int i = 0; i < kAux; ++i) {
      hipError_t e = xs_order(XS_JOIN0 + i, aux[i], stream);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // the store-update kernels' view of the dense state (dm_device.h DenseUpd)
  DenseUpd dense_upd() const {
    DenseUpd d{};
    d.item_of = item_of.p;
    for (int b = 3; b <= 6; ++b) d.bins[b - 3] = bins[b].p;
    d.bin4_wave = bin4_wave ? 1 : 0;
    d.bin6_wide = bin6_wide ? 1 : 0;
    d.rmask = rmask.p;
    return d;
  }
  // Queue calibration (calib_step): which of the four auxiliary streams -- four hardware
  // queues -- carries which work class moved configs[2]'s tick from 111 to 157 us over
  // the 24 assignments (profiles/r05_queues.txt), and a queue's place in the process's
  // creation order, which a host that made streams of its own first shifts, decides
  // which assignment is best.  So the context times every assignment on its first
  // forked writeback ticks (windows of kCalibWin ticks, each between joins of every
  // class stream, HIP events on the context stream), times the best kCalibFinal again
  // over longer windows, and keeps the fastest: aux[i] = aux_phys[perm[i]].
  // (the skip: a context's first ticks run slow -- first-touch, and the GPU reaches its
  // sustained-load operating point only after ~0.1-0.3 s of back-to-back work,
  // profiles/r06_c4_variants.md -- which biases the candidates timed first; round 2
  // therefore also interleaves its candidates, kCalibRep2 short windows each, and sums
  // them, so that a drift of the clocks falls on every candidate alike)
  static constexpr int kCalibSkip = 1024, kCalibWin = 6, kCalibFinal = 3, kCalibWin2 = 4, kCalibRep2 = 4;
  int calib = 0;  // 0 pending, 1 round 1, 2 round 2, 3 waiting for the events, 4 done / off
  int calib_skip = 0, calib_k = 0, calib_t = 0, calib_round = 0;
  int perm[kAux] = {0, 1, 2, 3};
  hipStream_t aux_phys[kAux] = {};
  std::vector<std::array<int, kAux>> calib_cand;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> calib_ev;
  std::vector<int> calib_of_ev;  // candidate timed by each window
  std::vector<float> calib_ms;
  bool calib_log = false;
  int64_t calib_best = -1;  // the chosen permutation (perm[0] + 4 perm[1] + 16 perm[2] + 64 perm[3])
  // plan
  std::vector<Tile> h_tiles;  // small resources (n <= kSmallMax) in tiles (k_tile_small)
  std::vector<TileEntry> h_tile_list;  // the list tiles' resources
  DBuf<TileEntry> tile_list;
  std::vector<WorkItem> h_bins[kNumBins];
  std::vector<Chunk> h_chunks;
  std::vector<LargeSeg> h_large;
  DBuf<Tile> tiles;
  DBuf<WorkItem> bins[kNumBins];
  DBuf<Chunk> chunks;
  DBuf<LargeSeg> large;
  // the sub-wave bins run in one launch (k_subs): C2 tick 144-145 -> 138 us against
  // one launch per bin (tools/ab.py, both orders, one box; the per-bin form was
  // retired in round 5)
  // The 128-thread bins (3, 4) split by the dense hint (k_block_dense + k_block_rest)
  // on a tick that follows a writeback tick (only those set hints), unless the last
  // split tick the host has heard of queued more than a quarter of the bin's items
  // for k_block_rest (then it tries again after 64 ticks, doubling the wait after every
  // try that still queued too many, up to 4096: C2's bins, whose resources keep
  // released rows, run 21 % slower split, and a try's k_block_rest strides over
  // thousands of items).  DM_DENSE_SPLIT=0: never split.
  int dense_split = 0xF;  // bit i: bin 3+i runs in the split form (DM_DENSE_SPLIT: 0 off, 1 all, else the mask)
  static constexpr int kSplitBins = 4;  // bins 3..6
  // Stream parts: a workgroup bin that is the store's only work class, and small enough
  // that a launch's ramp and drain are a visible share of it, runs as kParts launches
  // over contiguous halves of its items on two auxiliary streams, never joined from
  // tick to tick (DM_DEFER_JOIN): each part's next tick starts while the other part
  // drains, so the GPU never idles between ticks (an N = 8 shard of configs[3], 12.5M
  // leases: 57.3 -> 48.8 us per tick, tools/shard_split.py; the whole configs[3], 100M
  // leases: 430 -> 425 us, not worth its cross-queue waits in the exchange).  Every
  // split-bin state below is per part: slot (b - 3) * kParts + part.
  static constexpr int kParts = 2;
  static constexpr int kSplitSlots = kSplitBins * kParts;
  int bin_parts[kNumBins] = {1, 1, 1, 1, 1, 1, 1, 1, 1};
  // off for a leaf whose ticks an exchange on another stream waits for (dm_hier_attach):
  // there the exchange's two waits and the parts' CU share cost more than the parts
  // gain (the N = 8 rehearsal step 58.7 -> 66 us; one wait: 60-62 us; round 5)
  bool parts_ok = true;
  int64_t part_lo[kNumBins][kParts + 1] = {};  // item bounds of each part
  DBuf<int32_t> dq_list[kSplitSlots], dq_cnt[kSplitSlots];
  int dq_par[kSplitSlots] = {};
  int dq_skip[kSplitSlots] = {};   // ticks in the one-kernel form since the split was last tried
  int dq_wait[kSplitSlots] = {64, 64, 64, 64, 64, 64, 64, 64};  // ticks before the next try
  bool bin6_wide = false;  // bin 6 on 512 x 8 workgroups (kBin6Wide): it holds most of the rows
  bool bin4_wave = false;  // bin 4 on one wave per resource (kBin4Wave): most of its resources FairShare
  std::vector<int32_t> h_kind;  // the loaded configuration's kinds (bin 4's shape)
  int32_t* h_dq = nullptr;   // host-mapped: items the last split tick queued, per bin
  int32_t* d_dq = nullptr;
  // host-mapped, per split bin: {undense count, epoch} of the epoch's check
  // (k_count_undense), and the guard a dense kernel sets should it queue an item on a
  // tick whose rest kernel was skipped
  uint64_t* h_rec = nullptr;
  uint64_t* d_rec = nullptr;
  int32_t* h_guard = nullptr;
  int32_t* d_guard = nullptr;
  uint64_t dq_ver_epoch[kSplitSlots] = {};  // the epoch each slot's check was enqueued in
  // large-path partials
  DBuf<int64_t> pa_cnt, pa_cnt_all, pa_smin, pa_smax, pb_w, pc_sgt;
  DBuf<double> pa_has, pa_wants, pa_has_all, pa_wants_all, pb_x, pb_y, pc_ee, pd_delta;
  DBuf<int32_t> pa_nan;
  DBuf<uint32_t> pa_live;
  DBuf<uint8_t> p_tot;
  // the speculative chain (k_large_spec + k_large_redo; DM_SPEC_CHAIN=0: the chain):
  // per large resource its SpecTot, the redo's launch count, the host-mapped give-up flag
  bool spec_chain = true;
  DBuf<SpecTot> p_spec;
  DBuf<uint32_t> p_spec_ring;  // SpecArgs::ring
  // 3/4 of the redo workgroups (full build) the GPU holds at once: the full build's
  // grid when the store has that many team slots
  int64_t redo_cap = 0;
  // the redo by teams (k_large_redo_team): team slots and the two builds' grids.  (The
  // per-chunk redo of round 4, bounded by redo_cap chunks per resource, was retired in
  // round 5: the teams need only kTeamMax co-resident workgroups for any resource.)
  DBuf<int32_t> p_team;
  int nslots = 0, team_grid_full = 1, team_grid_light = 1;
  uint64_t spec_seq = 0;
  int32_t* h_serr = nullptr;  // [0] the give-up flag, [1] SpecArgs::seen
  int32_t* d_serr = nullptr;
  // k_large_redo's light build (dm_kernels.hip) while the last redo the host saw found
  // nothing marked and no row changed since (DM_REDO_LIGHT: 0 never, 1 so, 2 always)
  int redo_light = 1;
  uint64_t redo_epoch = 0;  // row_epoch at the last speculative tick
  DBuf<int32_t> p_uni;
  // heterogeneous FairShare on the chain (allocated on the first tick that may need it)
  DBuf<uint32_t> ph_set;  // per large resource: distinct subclient counts (all ones between ticks)
  DBuf<int32_t> ph_n, ph_bkc;
  size_t ph_set_ready = 0;  // large resources whose set slots are initialised
  DBuf<uint8_t> ph_het;
  DBuf<double> ph_bkw;
  DBuf<int64_t> ph_bks;
  // worklist of resources for k_general (heterogeneous-subclient FairShare)
  DBuf<int32_t> glist, gcount;
  bool maybe_general = false;
  bool all_sub_one = true;  // every loaded row had subclients == 1
  int64_t n_nonsmall = 0;
  // staging for upsert / release
  DBuf<int64_t> st_rows, st_sub, st_exp;
  DBuf<double> st_has, st_wants;
  DBuf<uint64_t> st_mask;  // dm_store_update_wants_mask
  DBuf<int64_t> st_blk;
  DBuf<int32_t> st_wpre;
  static constexpr int kWChunks = 4;  // dm_store_apply: the refresh values' copy chunks
  // One round's staging (dm_store_apply): set 0 for the synchronous call, sets 1..
  // kAsyncSets for dm_store_apply_async, whose batch k uses set 1 + k % kAsyncSets and is
  // retired (its flags read) before batch k + kAsyncSets reuses the set.
  struct ApplySet {
    DBuf<uint64_t> mask;
    DBuf<double> mwants;  // the refresh part's values
    DBuf<int64_t> blk;
    DBuf<int32_t> wpre;
    DBuf<int64_t> rel;  // the departures' rows
    DBuf<int64_t> rows, sub, exp;
    DBuf<double> has, wants;
    DBuf<uint32_t> flags;  // one flags word per part
    uint32_t* h_flags = nullptr;
    hipEvent_t ev_bat[3] = {};
    hipEvent_t ev_wchunk[kWChunks] = {};
    hipEvent_t ev_done = nullptr;  // (asynchronous sets) the batch's last kernel and flags copy
    bool pending = false;      // enqueued, not yet retired
    bool may_general = false;  // its refresh or arrivals may bring NaN wants / other subclient counts
    int64_t nu = 0;
    void release() {
      mask.release(); mwants.release(); blk.release(); wpre.release(); rel.release();
      rows.release(); sub.release(); exp.release(); has.release(); wants.release(); flags.release();
      if (h_flags) (void)hipHostFree(h_flags);
      h_flags = nullptr;
    }
    void destroy_events() {
      for (auto& ev : ev_bat) if (ev) { (void)hipEventDestroy(ev); ev = nullptr; }
      for (auto& ev : ev_wchunk) if (ev) { (void)hipEventDestroy(ev); ev = nullptr; }
      if (ev_done) (void)hipEventDestroy(ev_done);
      ev_done = nullptr;
    }
  };
  static constexpr int kAsyncSets = 2;
  ApplySet aset[1 + kAsyncSets];
  int64_t async_seq = 0;  // asynchronous batches enqueued
  // a tick enqueued while an asynchronous batch that may make the store general is in flight
  bool async_may_general() const {
    for (int i = 1; i <= kAsyncSets; ++i)
      if (aset[i].pending && aset[i].may_general) return true;
    return false;
  }
  DBuf<uint32_t> row_bits;     // device row bitmap for the uniqueness check, all-zero between calls
  DBuf<uint32_t> upd_flags;    // k_check_rows result (device)
  // dm_decide: a round's requests (grouped by resource), per-resource work items, results
  DBuf<int64_t> rq_rows, rq_sub, rq_exp;
  DBuf<double> rq_has, rq_wants, rq_gets;
  DBuf<ReqItem> rq_items;
  DBuf<double> rq_sc_has, rq_sc_wants;  // the round's working copy of the requested resources' rows
  DBuf<int32_t> rq_sc_sub;
  // dm_decide's fast path (dm_decide_fast.hip); DM_DECIDE_FAST=0 turns it off
  bool decide_fast = true;
  DBuf<FastItem> fd_items;
  DBuf<FastRes> fd_res;
  DBuf<int64_t> fd_prev, fd_bounds;
  DBuf<double> fd_pw, fd_v, fd_keys, fd_keys_s, fd_ev_in, fd_ev;
  DBuf<FdScan> fd_sc, fd_ps, fd_part;
  DBuf<int32_t> fd_evs_in, fd_evs, fd_ecnt, fd_bdc;
  DBuf<double2> fd_esum, fd_bds;
  DBuf<FdClean> fd_pc;
  DBuf<FdScan> fd_pt;
  DBuf<FdLind> fd_ld;
  DBuf<uint8_t> fd_tmp;
  // dm_publish_totals: the workgroups' validation flags and their arrival counter
  // (k_publish; both return to zero after each launch)
  DBuf<uint32_t> pub_sync;
  // dm_publish_ring: writeback tick k publishes into pub_ring[k % n]
  std::vector<double2*> pub_ring;
  int64_t pub_k = 0;
  // root side of the hierarchy: the exchange's layout (dm_hier_layout) and the
  // last round's per-server flags
  int hier_G = 0;                    // 0: not configured (replicated, G from each call)
  bool hier_sharded = false;
  std::vector<int64_t> h_hier_lo;    // [G + 1] sharded bounds
  DBuf<int64_t> hier_lo;
  int64_t hier_stride = 0;
  DBuf<uint32_t> hier_status;
  int hier_servers = 0;
  // dm_hier_attach / dm_hier_step (root side): the leaf it serves, its ring and gathered
  // buffer, its server index; the exchange's RCCL communicator (dm_hier_comm_init)
  dm_ctx* hs_leaf = nullptr;
  int hs_server = 0;
  std::vector<void*> hs_ring;
  void* hs_gathered = nullptr;
  ncclComm_t nccl_comm = nullptr;
  bool hs_ordered = false;  // dm_hier_step already ordered the exchange stream after the tick
  // leaf side: pipelined templates (dm_hier_pipeline).  An exchange stages this
  // leaf's new templates in a free slot; the leaf's ticks take the staged templates
  // of the exchanges enqueued before the previous tick (one tick of lag).
  bool tpl_pipe = false;
  int tpl_lag = 1;  // ticks between an exchange and the first tick that takes its templates, minus one
  DBuf<ResCfg> tpl_cfg[kTplSlots];
  DBuf<ResCold> tpl_cold[kTplSlots];
  XsTok tpl_ready[kTplSlots];        // root stream: the slot's templates are written
  XsTok tpl_free[kTplSlots];         // leaf stream: the ticks that read the slot are done
  bool tpl_free_rec[kTplSlots] = {};  // tpl_free holds a signal
  struct Staged {
    int slot;
    int64_t tag;  // leaf ticks issued before the exchange was enqueued
  };
  std::vector<Staged> tpl_pending;          // oldest first
  std::vector<int> tpl_free_slots;
  int64_t ticks_issued = 0;
  // The tick-done signal: ticks numbered by tick_seq (never reset).  The last kernel of
  // a one-class split tick (C1, C3: the dense kernel, or the rest kernel after it) is
  // launched with a stop event (hipExtLaunchKernel: the kernel's own completion signal,
  // no marker packet of its own on the leaf's queue -- each marker cost a ~10-us bubble
  // per N = 8 shard step), one event per tick in a ring; another queue waits on it.
  // Round 4 stored a word from a one-wave k_tick_done after the dense kernel (5 us of
  // the leaf's queue): the N = 8 rehearsal step 60.2-60.7 -> 58.7-58.8 us (round 5,
  // gpurun_out/r5b2shard, three alternations).
  // The event covers the tick's leases and sums, not every launch of it: once per row
  // epoch a writeback tick enqueues k_count_undense after the event-carrying kernel on
  // the same stream (check_dense).  That kernel only reads the work items' hints and
  // writes a host-mapped count, which no consumer of the event (the exchange, a template
  // slot's reuse) touches; a consumer that needed it would have to join the stream.
  uint64_t tick_seq = 0;          // the last tick's number
  bool tick_flagged = false;      // ... and whether its last kernels complete tick_ev[*][tick_seq % kTickEv]
  static constexpr int kTickEv = 16;
  hipEvent_t tick_ev[kParts][kTickEv] = {};  // per stream part (one part: [0])
  int tick_nev[kTickEv] = {};                // the parts that completed each flagged tick's events
  unsigned tick_part_mask = 0;               // auxiliary streams of the last flagged tick's parts
  // auxiliary streams with work not yet joined into the context stream
  unsigned aux_unjoined = 0;
  // the last tick's events cover every auxiliary stream's unjoined work, so a consumer
  // may wait on them instead of joining (which would make the next tick's parts wait
  // for each other: 49 -> 74 us per tick on the N = 8 shard, tools/shard_split.py)
  bool tick_covers() const { return tick_flagged && tick_part_mask != 0 && (aux_unjoined & ~tick_part_mask) == 0; }
  // a stream part's auxiliary stream (part 0: the bin's class stream).  Part 1 beside
  // bins 4-6's stream 1: stream 2 or 0 run C1 at 40.6-40.8 us per tick, stream 3 at
  // 61.6-64.2 us (which hardware queues pair well: take_aux; profiles/r05_parts_ab.txt)
  int part_stream(int b, int j) const {
    if (j == 0) return class_stream[b];
    return class_stream[b] != 2 ? 2 : 0;
  }
  // set by the first consumer on another stream (the exchange's order, a template
  // slot's reuse): before it, no tick carries the event
  bool tick_signal_wanted = false;
  uint64_t tpl_free_seq[kTplSlots] = {};  // a slot is free once this tick's event completed (0: use tpl_free)
  uint32_t* h_flags = nullptr; // pinned host mirror of upd_flags
  // profiling
  bool profiling = false;
  std::vector<ProfEvent> pending;
  std::vector<hipEvent_t> event_pool;
  int64_t prof_launches[KC_COUNT] = {};
  double prof_ms[KC_COUNT] = {};

  int fail(int code, const std::string& msg) {
    err = msg;
    g_last_error = msg;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    return fail(DM_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  }
  // The device's failure words (host-mapped, written by kernels of earlier ticks):
  // once one is set the store is lost (store_lost).  Called at the entry of every call
  // that touches the store and after every host wait that may have completed a tick.
  int check_device() {
    if (!store_lost) {
      for (int i = 0; h_guard && i < kSplitSlots; ++i)
        if (__atomic_load_n(h_guard + i, __ATOMIC_RELAXED)) {
          store_lost = true;
          lost_msg = "a dense kernel queued an item on a tick that skipped its rest kernel";
        }
      if (!store_lost && h_serr && __atomic_load_n(h_serr, __ATOMIC_RELAXED)) {
        store_lost = true;
        lost_msg = "a redo workgroup of the speculative chain gave up waiting for its resource";
      }
    }
    if (!store_lost || reading) return DM_OK;  // (a reader of a lost store: dm_store_lost says so)
    return fail(DM_E_INTERNAL, "internal failure on the device: " + lost_msg +
                                   "; the store's leases and sums may be wrong, reload it (dm_store_load)");
  }
  bool reading = false;  // a read call in progress (DM_STORE_READABLE): a lost store may be read
  // wait for the context stream, then report a device failure the wait completed
  int synced(const char* what) {
    const hipError_t e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_fail(e, what);
    return check_device();
  }
  hipEvent_t take_event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  // HIP events around one launch on its stream while profiling is on (dm_kernel_times)
  template <typename F>
  hipError_t timed(int cls, hipStream_t s, F&& fn) {
    if (!profiling) return fn();
    ProfEvent pe{cls, take_event(), take_event()};
    (void)hipEventRecord(pe.a, s);
    hipError_t e = fn();
    (void)hipEventRecord(pe.b, s);
    pending.push_back(pe);
    return e;
  }
  void collect_profile() {
    for (auto& pe : pending) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
        prof_ms[pe.cls] += ms;
        prof_launches[pe.cls] += 1;
      }
      event_pool.push_back(pe.a);
      event_pool.push_back(pe.b);
    }
    pending.clear();
  }
  void free_all() {
    seg_off.release(); blk_seg.release(); wants.release(); has.release(); sub.release(); expiry.release();
    agg.release(); expl.release(); cfg.release(); cold.release();
    out_gets.release(); out_expiry.release(); res.release();
    tiles.release(); for (auto& b : bins) b.release(); chunks.release(); large.release();
    for (int i = 0; i < kSplitSlots; ++i) {
      dq_list[i].release();
      dq_cnt[i].release();
    }
    if (h_dq) (void)hipHostFree(h_dq);
    h_dq = nullptr;
    d_dq = nullptr;
    if (h_rec) (void)hipHostFree(h_rec);
    h_rec = d_rec = nullptr;
    if (h_guard) (void)hipHostFree(h_guard);
    h_guard = d_guard = nullptr;
    pa_cnt.release(); pa_cnt_all.release(); pa_has_all.release(); pa_wants_all.release(); pa_smin.release(); pa_smax.release(); pb_w.release(); pc_sgt.release();
    pa_has.release(); pa_wants.release(); pb_x.release(); pb_y.release(); pc_ee.release(); pd_delta.release();
    pa_nan.release(); pa_live.release(); p_tot.release(); p_uni.release(); p_spec.release(); p_spec_ring.release(); p_team.release();
    if (h_serr) (void)hipHostFree(h_serr);
    h_serr = d_serr = nullptr;
    ph_set.release(); ph_n.release(); ph_bkc.release(); ph_het.release(); ph_bkw.release(); ph_bks.release();
    ph_set_ready = 0;
    glist.release(); gcount.release();
    st_rows.release(); st_sub.release(); st_exp.release(); st_has.release(); st_wants.release();
    st_mask.release(); st_blk.release(); st_wpre.release();
    for (auto& a : aset) {
      a.release();
      a.pending = false;
    }
    row_bits.release(); upd_flags.release(); hier_status.release(); hier_lo.release(); pub_sync.release();
    for (int i = 0; i < kTplSlots; ++i) {
      tpl_cfg[i].release();
      tpl_cold[i].release();
    }
    rq_rows.release(); rq_sub.release(); rq_exp.release(); rq_has.release(); rq_wants.release(); rq_gets.release();
    rq_items.release(); rq_sc_has.release(); rq_sc_wants.release(); rq_sc_sub.release();
    fd_items.release(); fd_res.release(); fd_prev.release(); fd_bounds.release(); fd_pw.release(); fd_v.release();
    fd_keys.release(); fd_keys_s.release(); fd_ev_in.release(); fd_ev.release(); fd_sc.release(); fd_ps.release();
    fd_part.release(); fd_evs_in.release(); fd_evs.release(); fd_ecnt.release(); fd_bdc.release(); fd_esum.release();
    fd_bds.release(); fd_tmp.release(); fd_pc.release(); fd_pt.release(); fd_ld.release();
    if (h_flags) (void)hipHostFree(h_flags);
    h_flags = nullptr;
  }
};

#define DM_HIP(ctx, expr, what)                  \
  do {                                           \
    hipError_t _e = (expr);                      \
    if (_e != hipSuccess) return (ctx)->hip_fail(_e, what); \
  } while (0)

#define DM_CHECK_CTX(ctx)                                   \
  do {                                                      \
    if (!(ctx)) {                                           \
      g_last_error = "null context";                        \
      return DM_E_INVAL;                                    \
    }                                                       \
    DM_HIP(ctx, hipSetDevice((ctx)->device), "hipSetDevice"); \
  } while (0)

// Entry of every call that puts work on the context stream: join the auxiliary
// streams' deferred tick work first (DM_DEFER_JOIN), and remember that the
// context stream now holds work the next fork must order.
#define DM_ENTER(ctx)                                         \
  do {                                                        \
    DM_CHECK_CTX(ctx);                                        \
    DM_HIP(ctx, (ctx)->join_aux(), "join auxiliary streams"); \
    (ctx)->main_dirty = true;                                 \
  } while (0)

// Entry of every call that reads or updates the store: refuse a lost store
// (dm_ctx::store_lost) with the device's message.
#define DM_STORE_OK(ctx)                             \
  do {                                               \
    if (int _rc = (ctx)->check_device()) return _rc; \
  } while (0)
// The read calls work on a lost store too (for diagnosis): the failure is
// still recorded, and dm_store_lost reports it.  Ticks and updates keep refusing it.
struct ReadScope {
  dm_ctx* c;
  explicit ReadScope(dm_ctx* x) : c(x) { c->reading = true; }
  ~ReadScope() { c->reading = false; }
};
#define DM_STORE_READABLE(ctx)  \
  ReadScope _read_scope(ctx); \
  (void)(ctx)->check_device()

template <typename T>
static hipError_t upload(DBuf<T>& b, const T* src, size_t n, hipStream_t st) {
  hipError_t e = b.ensure(n);
  if (e != hipSuccess || n == 0) return e;
  return hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, st);
}

// ---------------------------------------------------------------------------
// plan: size-binned dispatch
// ---------------------------------------------------------------------------
static int bin_of(int64_t n) {
  if (n <= 16) return 7;
  if (n <= 32) return 8;
  if (n <= 64) return 0;
  if (n <= 128) return 1;
  if (n <= 256) return 2;
  if (n <= 512) return 3;
  if (n <= 1024) return 4;
  if (n <= 2048) return 5;
  return 6;
}

static void build_plan(dm_ctx* c) {
  c->h_tiles.clear();
  for (auto& b : c->h_bins) b.clear();
  c->h_chunks.clear();
  c->h_large.clear();
  const std::vector<int64_t>& off = c->h_seg_off;
  std::vector<int64_t> large;
  c->h_tile_list.clear();
  // runs of at least kTileMinRun consecutive small resources: tiles of at most kTileRes
  // resources and kTileRows rows; the small resources of shorter runs: list tiles
  std::vector<int32_t> scattered;
  auto run_tiles = [&](int64_t r0, int64_t r1) {
    if (r1 - r0 < kTileMinRun) {
      for (int64_t r = r0; r < r1; ++r) scattered.push_back((int32_t)r);
      return;
    }
    Tile tc{};
    bool topen = false;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t n = off[r + 1] - off[r];
      if (topen && (tc.nrows + n > kTileRows || tc.nseg >= kTileRes)) {
        c->h_tiles.push_back(tc);
        topen = false;
      }
      if (!topen) {
        tc = Tile{(int32_t)r, 0, off[r], 0, 0};
        topen = true;
      }
      tc.nseg += 1;
      tc.nrows += (int32_t)n;
    }
    if (topen) c->h_tiles.push_back(tc);
  };
  int64_t run0 = -1;
  for (int64_t r = 0; r < c->R; ++r) {
    const int64_t n = off[r + 1] - off[r];
    if (n <= kSmallMax) {
      if (run0 < 0) run0 = r;
      continue;
    }
    if (run0 >= 0) run_tiles(run0, r);
    run0 = -1;
    if (n <= kLargeMin) {
      c->h_bins[bin_of(n)].push_back(WorkItem{(int32_t)r, (int32_t)n, off[r]});
    } else {
      large.push_back(r);
    }
  }
  if (run0 >= 0) run_tiles(run0, c->R);
  static_assert(kTileRes * kSmallMax <= kTileRows, "a list tile of kTileRes resources fits its LDS rows");
  for (size_t i = 0; i < scattered.size(); i += kTileRes) {
    const size_t e = std::min(scattered.size(), i + (size_t)kTileRes);
    Tile tc{(int32_t)c->h_tile_list.size(), (int32_t)(e - i), 0, 0, 1};
    for (size_t j = i; j < e; ++j) {
      const int32_t r = scattered[j];
      c->h_tile_list.push_back(TileEntry{r, tc.nrows});
      tc.nrows += (int32_t)(off[(size_t)r + 1] - off[(size_t)r]);
    }
    c->h_tiles.push_back(tc);
  }
  // the sub-wave bins: items ordered by shape (the narrowest kSubShapeG x kSubShapeR
  // that holds the resource, dm_device.h), each shape's items in resource order
  for (int k = 0; k < kSubShapes; ++k) {
    const int b = kSubShapeBin[k];
    const bool first = k == 0 || kSubShapeBin[k - 1] != b;
    const int64_t lo = first ? 0 : c->h_shape_lo[k - 1] + c->h_shape_n[k - 1];
    std::vector<WorkItem>& v = c->h_bins[b];
    const int cap = kSubShapeG[k] * kSubShapeR[k];
    auto mid = std::stable_partition(v.begin() + lo, v.end(), [&](const WorkItem& w) { return (w.n & 0xFFFF) <= cap; });
    c->h_shape_lo[k] = lo;
    c->h_shape_n[k] = (int64_t)(mid - v.begin()) - lo;
  }
  // Large resources largest first: a resource is verified by its last-arriving chunk,
  // and the largest's verification (the longest canonical trees) then overlaps the
  // other chunks instead of trailing the launch.  Each resource's chunks stay
  // consecutive and in row order (the canonical trees' order).
  std::stable_sort(large.begin(), large.end(),
                   [&](int64_t a, int64_t b) { return off[a + 1] - off[a] > off[b + 1] - off[b]; });
  for (const int64_t r : large) {
    LargeSeg L{(int32_t)r, (int32_t)c->h_chunks.size(), 0, 0};
    for (int64_t o = off[r]; o < off[r + 1]; o += kChunkRows) {
      Chunk ch{(int32_t)r, (int32_t)c->h_large.size(), o, (int32_t)std::min<int64_t>(kChunkRows, off[r + 1] - o), 0};
      c->h_chunks.push_back(ch);
    }
    L.chunk_end = (int32_t)c->h_chunks.size();
    c->h_large.push_back(L);
  }
}

// Once per row epoch, after a writeback tick of workgroup bin b's part j (split slot
// i): count its items left without a dense hint (k_count_undense -> h_rec).  A count
// of 0 lets the following ticks of the epoch skip the part's k_block_rest.
static hipError_t check_dense(dm_ctx* c, int i, int b, int j, hipStream_t s) {
  const int64_t lo = c->part_lo[b][j], n = c->part_lo[b][j + 1] - lo;
  if (c->dq_ver_epoch[i] == c->row_epoch || n <= 0) return hipSuccess;
  c->dq_ver_epoch[i] = c->row_epoch;
  return launch_count_undense(c->bins[b].p + lo, (int)n, (unsigned long long*)(c->d_rec + 2 * i),
                              (unsigned long long)c->row_epoch, s);
}

// The auxiliary stream of each launch unit of a tick (the sub-wave launch of bins 7, 8,
// 0, 1, 2; the workgroup bins 3-6, each a launch; the small tiles; the large chain).
// dm_ctx::kClassStream is the measured assignment for a store holding every class
// (configs[2]: bins 3-6 share stream 1 with bin 3 beside the sub-wave launch on stream 2,
// all hidden behind the large chain's critical path).  A store holding only some classes
// (a resource-id shard of a Zipf population: the head shards hold the large and
// workgroup classes, the tail shards the small ones) would then run classes one after
// another on a shared stream while another stream idles: the N = 8 shard of bins 3-6
// ran 36.6 us against 24-26 for its neighbours (profiles/r06_c2_shard8_ranks_contiguous_before_stream_plan.json).
// So, while some stream holds no unit of this store, the largest unit (by rows and
// records) of a stream holding several moves to it.
static void plan_streams(dm_ctx* c) {
  for (int i = 0; i < kNumBins + 2; ++i) c->class_stream[i] = dm_ctx::kClassStream[i];
  for (int b = 0; b < kNumBins; ++b)
    if (c->bin_parts[b] > 1) return;  // one bin in stream parts: its own two streams
  constexpr int kUnits = 7;  // 0 sub-wave launch, 1-4 bins 3-6, 5 tiles, 6 large chain
  auto unit_of_bin = [](int b) { return (b >= 3 && b <= 6) ? b - 2 : 0; };
  double bytes[kUnits] = {};
  bool present[kUnits] = {};
  const std::vector<int64_t>& off = c->h_seg_off;
  for (int b = 0; b < kNumBins; ++b)
    for (const WorkItem& w : c->h_bins[b]) {
      present[unit_of_bin(b)] = true;
      bytes[unit_of_bin(b)] += 28.0 * (double)(off[(size_t)w.seg + 1] - off[(size_t)w.seg]) + 97.0;
    }
  for (const Tile& t : c->h_tiles) {
    present[5] = true;
    bytes[5] += 28.0 * t.nrows + 97.0 * t.nseg;
  }
  for (const LargeSeg& L : c->h_large) {
    present[6] = true;
    bytes[6] += 28.0 * (double)(off[(size_t)L.seg + 1] - off[(size_t)L.seg]) + 97.0;
  }
  int us[kUnits];
  for (int u = 0; u < kUnits; ++u) us[u] = dm_ctx::kClassStream[u == 0 ? 0 : u <= 4 ? u + 2 : u == 5 ? kNumBins : kNumBins + 1];
  for (;;) {
    int load[dm_ctx::kAux] = {};
    for (int u = 0; u < kUnits; ++u) load[us[u]] += present[u] ? 1 : 0;
    int idle = -1, mover = -1;
    for (int k = 0; k < dm_ctx::kAux && idle < 0; ++k)
      if (load[k] == 0) idle = k;
    for (int u = 0; u < kUnits; ++u)
      if (present[u] && load[us[u]] > 1 && (mover < 0 || bytes[u] > bytes[mover])) mover = u;
    if (idle < 0 || mover < 0) break;
    us[mover] = idle;
  }
  for (int b = 0; b < kNumBins; ++b) c->class_stream[b] = us[unit_of_bin(b)];
  c->class_stream[kNumBins] = us[5];
  c->class_stream[kNumBins + 1] = us[6];
}

// Stream parts (dm_ctx::kParts): a workgroup bin holding every resource of the store
// (no other bin, tile or chunk, no heterogeneous subclients) and at most kPartBytes of
// rows, with enough items that each half still fills the GPU.
constexpr int64_t kPartBytes = int64_t(1) << 30;
constexpr int64_t kPartMinItems = 4096;
static void plan_parts(dm_ctx* c) {
  int nonempty = 0, only = -1;
  for (int b = 0; b < kNumBins; ++b)
    if (!c->h_bins[b].empty()) {
      ++nonempty;
      only = b;
    }
  for (int b = 0; b < kNumBins; ++b) {
    const int64_t n = (int64_t)c->h_bins[b].size();
    const bool split = c->parts_ok && nonempty == 1 && only == b && b >= 3 && b < 3 + dm_ctx::kSplitBins && c->h_tiles.empty() &&
                       c->h_chunks.empty() && !c->maybe_general && n >= kPartMinItems && c->N * 28 <= kPartBytes;
    c->bin_parts[b] = split ? dm_ctx::kParts : 1;
    for (int j = 0; j <= dm_ctx::kParts; ++j)
      c->part_lo[b][j] = split ? n * j / dm_ctx::kParts : (j == 0 ? 0 : n);
  }
  plan_streams(c);
}

// kBin4Wave (dm_device.h): bin 4 in stream parts and most of its resources FairShare
// by the loaded kinds.  (Without parts the shape did not pay: configs[3]'s N = 8 shard
// and the whole configs[3] unchanged, its N = 4 shard +3 %, profiles/r05_ab/b4_one_wave.txt.)
static bool bin4_prefers_wave(const dm_ctx* c) {
  const std::vector<WorkItem>& items = c->h_bins[4];
  if (items.empty() || c->bin_parts[4] < 2 || (int64_t)c->h_kind.size() != c->R) return false;
  int64_t fs = 0;
  for (const WorkItem& w : items) fs += c->h_kind[(size_t)w.seg] == DM_FAIR_SHARE ? 1 : 0;
  return 2 * fs > (int64_t)items.size();
}

// Bin 4's shape after a new plan, new kinds or parts turned off: a change re-uploads the
// bin's items without their hints (the dense hints and released-row masks are the
// shape's own; the next writeback tick sets them in the new shape).
static int update_bin4_shape(dm_ctx* c, hipStream_t st) {
  const bool wave = bin4_prefers_wave(c);
  if (wave == c->bin4_wave) return DM_OK;
  c->bin4_wave = wave;
  DM_HIP(c, upload(c->bins[4], c->h_bins[4].data(), c->h_bins[4].size(), st), "plan bins");
  return DM_OK;
}

// The stream parts of the plan and every split slot's state: rest queues, two-slot
// counters, the epoch checks (a new plan, or parts turned off).
static int init_split_slots(dm_ctx* c, hipStream_t st) {
  plan_parts(c);
  for (int i = 0; i < dm_ctx::kSplitSlots; ++i) {
    __atomic_store_n(c->h_rec + 2 * i + 1, (uint64_t)0, __ATOMIC_RELAXED);
    __atomic_store_n(c->h_guard + i, 0, __ATOMIC_RELAXED);
    c->dq_ver_epoch[i] = 0;
    __atomic_store_n(c->h_dq + i, 0, __ATOMIC_RELAXED);
    c->dq_skip[i] = 0;
    c->dq_wait[i] = 64;
    const int b = 3 + i / dm_ctx::kParts, j = i % dm_ctx::kParts;
    const size_t nb = (size_t)std::max<int64_t>(c->part_lo[b][j + 1] - c->part_lo[b][j], 1);
    DM_HIP(c, c->dq_list[i].ensure(nb), "dense split queue");
    DM_HIP(c, c->dq_cnt[i].ensure(3), "dense split queue");  // two-slot count + the last count told the host
    DM_HIP(c, hipMemsetAsync(c->dq_cnt[i].p, 0, 3 * sizeof(int32_t), st), "dense split queue");
    c->dq_par[i] = 0;
  }
  return DM_OK;
}

// Stream parts allowed or not (dm_ctx::parts_ok): the plan's parts and the split slots
// are set up again after every stream has drained.
static int set_parts_ok(dm_ctx* c, bool ok) {
  if (c->parts_ok == ok) return DM_OK;
  c->parts_ok = ok;
  if (!c->h_dq) return DM_OK;  // no plan yet: upload_plan reads the flag
  DM_HIP(c, c->join_aux(), "join");
  if (int rc = c->synced("stream parts")) return rc;
  c->main_dirty = true;
  if (int rc = init_split_slots(c, c->stream)) return rc;
  return update_bin4_shape(c, c->stream);
}

static int upload_plan(dm_ctx* c) {
  hipStream_t st = c->stream;
  DM_HIP(c, upload(c->tiles, c->h_tiles.data(), c->h_tiles.size(), st), "plan tiles");
  DM_HIP(c, upload(c->tile_list, c->h_tile_list.data(), c->h_tile_list.size(), st), "plan tiles");
  for (int b = 0; b < kNumBins; ++b) DM_HIP(c, upload(c->bins[b], c->h_bins[b].data(), c->h_bins[b].size(), st), "plan bins");
  {  // every workgroup-bin resource's item (the update kernels keep its dense state, DenseUpd)
    std::vector<int32_t> io((size_t)std::max<int64_t>(c->R, 1), -1);
    for (int b = 3; b <= 6; ++b)
      for (size_t i = 0; i < c->h_bins[b].size(); ++i) io[(size_t)c->h_bins[b][i].seg] = (int32_t)(b << 24 | (int)i);
    DM_HIP(c, upload(c->item_of, io.data(), io.size(), st), "plan items");
    // the masks of a new plan start empty (the arrival masks are read only where an upsert
    // set a bit; the released-row masks are written whole when a tick sets the dense state)
    DM_HIP(c, hipMemsetAsync(c->rmask.p, 0, c->rmask.n, st), "plan masks");
  }
  DM_HIP(c, upload(c->chunks, c->h_chunks.data(), c->h_chunks.size(), st), "plan chunks");
  DM_HIP(c, upload(c->large, c->h_large.data(), c->h_large.size(), st), "plan large");
  if (!c->h_dq) {
    // fine-grained (coherent) host memory: a device store lands in host memory at once,
    // not in the GPU's L2 until a system-scope release (which a profiled dispatch under
    // rocprofv3 need not issue: the rest-skip check was never seen there)
    DM_HIP(c, hipHostMalloc((void**)&c->h_dq, dm_ctx::kSplitSlots * sizeof(int32_t),
                            hipHostMallocMapped | hipHostMallocCoherent),
           "dense split word");
    DM_HIP(c, hipHostGetDevicePointer((void**)&c->d_dq, c->h_dq, 0), "dense split word");
    DM_HIP(c, hipHostMalloc((void**)&c->h_rec, dm_ctx::kSplitSlots * 2 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent),
           "dense split check");
    DM_HIP(c, hipHostGetDevicePointer((void**)&c->d_rec, c->h_rec, 0), "dense split check");
    DM_HIP(c, hipHostMalloc((void**)&c->h_guard, dm_ctx::kSplitSlots * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent),
           "dense split guard");
    DM_HIP(c, hipHostGetDevicePointer((void**)&c->d_guard, c->h_guard, 0), "dense split guard");
  }
  c->rows_changed();  // new work items: no hints
  {
    int64_t rows6 = 0;
    for (const WorkItem& w : c->h_bins[6]) rows6 += w.n & 0xFFFF;
    c->bin6_wide = 2 * rows6 > c->N;
  }
  if (int rc = init_split_slots(c, st)) return rc;
  if (int rc = update_bin4_shape(c, st)) return rc;
  const size_t nc = std::max<size_t>(c->h_chunks.size(), 1);
  DM_HIP(c, c->pa_cnt.ensure(nc), "partials");
  DM_HIP(c, c->pa_cnt_all.ensure(nc), "partials");
  DM_HIP(c, c->pa_has_all.ensure(nc), "partials");
  DM_HIP(c, c->pa_wants_all.ensure(nc), "partials");
  DM_HIP(c, c->pa_smin.ensure(nc), "partials");
  DM_HIP(c, c->pa_smax.ensure(nc), "partials");
  DM_HIP(c, c->pb_w.ensure(nc), "partials");
  DM_HIP(c, c->pc_sgt.ensure(nc), "partials");
  DM_HIP(c, c->pa_has.ensure(nc), "partials");
  DM_HIP(c, c->pa_wants.ensure(nc), "partials");
  DM_HIP(c, c->pb_x.ensure(nc), "partials");
  DM_HIP(c, c->pb_y.ensure(nc), "partials");
  DM_HIP(c, c->pc_ee.ensure(nc), "partials");
  DM_HIP(c, c->pd_delta.ensure(nc), "partials");
  DM_HIP(c, c->pa_nan.ensure(nc), "partials");
  DM_HIP(c, c->pa_live.ensure(nc * 256), "partials");
  DM_HIP(c, c->p_uni.ensure(nc), "partials");
  DM_HIP(c, c->p_tot.ensure(std::max<size_t>(c->h_large.size(), 1) * kSegTotBytes), "partials");
  {  // no resource has totals to speculate on yet (valid 0)
    const size_t nl = std::max<size_t>(c->h_large.size(), 1);
    DM_HIP(c, c->p_spec.ensure(nl), "speculative chain");
    DM_HIP(c, hipMemsetAsync(c->p_spec.p, 0, nl * sizeof(SpecTot), st), "speculative chain");
    DM_HIP(c, c->p_spec_ring.ensure(4), "speculative chain");
    DM_HIP(c, hipMemsetAsync(c->p_spec_ring.p, 0, 4 * sizeof(uint32_t), st), "speculative chain");
    std::vector<int32_t> team;
    for (size_t l = 0; l < c->h_large.size(); ++l) {
      const int nch_l = c->h_large[l].chunk_end - c->h_large[l].chunk_begin;
      for (int m = 0; m < std::min(nch_l, kTeamMax); ++m) team.push_back((int32_t)(l << 8 | (size_t)m));
    }
    c->nslots = (int)team.size();
    DM_HIP(c, upload(c->p_team, team.data(), team.size(), st), "redo teams");
    // every team's members can be resident at once: >= kTeamMax workgroups (the full
    // build: up to what the GPU holds; the light one: a steady tick's launch is all it costs)
    c->team_grid_full = std::max(1, (int)std::min<int64_t>(c->nslots, std::max<int64_t>(kTeamMax, c->redo_cap)));
    c->team_grid_light = std::max(1, std::min(c->nslots, kTeamMax));
    c->spec_seq = 0;
    if (!c->h_serr) {
      DM_HIP(c, hipHostMalloc((void**)&c->h_serr, 2 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent),
             "speculative chain");
      DM_HIP(c, hipHostGetDevicePointer((void**)&c->d_serr, c->h_serr, 0), "speculative chain");
    }
    __atomic_store_n(c->h_serr, 0, __ATOMIC_RELAXED);
    __atomic_store_n(c->h_serr + 1, 1, __ATOMIC_RELAXED);  // no redo seen yet: the full build first
  }
  DM_HIP(c, hipMemsetAsync(c->p_tot.p, 0, std::max<size_t>(c->h_large.size(), 1) * kSegTotBytes, st),
         "partials");  // SegTot::rel starts clear
  c->n_nonsmall = 0;
  for (int64_t r = 0; r < c->R; ++r)
    if (c->h_seg_off[r + 1] - c->h_seg_off[r] > kSmallMax) ++c->n_nonsmall;
  DM_HIP(c, c->glist.ensure((size_t)std::max<int64_t>(c->n_nonsmall, 1)), "worklist");
  DM_HIP(c, c->gcount.ensure(1), "worklist");
  return DM_OK;
}

// Could some non-small resource need k_general (heterogeneous subclients or NaN
// wants among its rows)?  Conservative: expiry is ignored.
// Could any FairShare resource need k_general (live subclients not all equal, or NaN
// wants)?  Released rows (DM_RELEASED) are never live, so they do not count.
static bool scan_maybe_general(const int64_t* off, int64_t R, const int64_t* sub, const double* wants,
                               const int64_t* exp) {
  for (int64_t r = 0; r < R; ++r) {
    if (off[r + 1] - off[r] <= kSmallMax) continue;
    int64_t s0 = -1;
    for (int64_t i = off[r]; i < off[r + 1]; ++i) {
      if (exp[i] == DM_RELEASED) continue;
      if (std::isnan(wants[i])) return true;
      if (s0 < 0) s0 = sub[i];
      if (sub[i] != s0) return true;
    }
  }
  return false;
}

template <typename T>
static hipError_t download(T* dst, const T* src, int64_t off, int64_t n, hipStream_t st) {
  if (!dst || n == 0) return hipSuccess;
  return hipMemcpyAsync(dst, src + off, (size_t)n * sizeof(T), hipMemcpyDeviceToHost, st);
}


// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* dm_version(void) { return "doorman-hip 0.6 (gfx950, abi 6)"; }

int dm_device_count(int* out) {
  if (!out) return DM_E_INVAL;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    g_last_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
    *out = 0;
    return DM_E_HIP;
  }
  *out = n;
  return DM_OK;
}

// The context's cross-stream order (dm_ctx::xs_signal): one event per hop kind.
static hipError_t xs_setup(dm_ctx* c) {
  for (int i = 0; i < dm_ctx::XS_N; ++i) {
    hipError_t e = hipEventCreateWithFlags(&c->xs_ev[i], hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The context's streams (its own stream, the four auxiliary streams, the copy stream),
// kept for the life of the process and reused by later contexts on the same device
// (dm_destroy returns a context's set; take_aux hands out the earliest-created free
// set).  The hardware queues behind the streams are not interchangeable: measured on
// C2 (round 5, tools/archive/gpu_r5_perm.sh, profiles/r05_queues.txt), which of the four
// masked queues carries which work class moved the tick from 111 us to 157 us, and the
// best assignment is a property of the queue's position in the process's creation
// order (period 4, consistent with queues spread over four hardware pipes): the small
// tiles on the last-created queue, every other assignment with the tiles elsewhere
// 123-157 us.  Stream priority does not change it.  So the creation order below is
// part of the tuning (own stream, the four masked streams, then the copy stream:
// 110-112 us; the copy stream first 137 us; the masked streams first 125 us), and a
// set is reused rather than destroyed and created again: new queues take other
// positions (bench.py's default run measured configs[2] at 124-154 us after earlier
// contexts were destroyed, 111-113 us with the pool).
struct AuxSet {
  int device;
  uint64_t seq;  // creation order: the earliest set first (its queues' positions, below)
  hipStream_t s[dm_ctx::kAux];
  hipStream_t own, cpy;  // the context's own stream and its copy stream, pooled with them
  bool own_queue;  // every stream got its own hardware queue (CU mask)
};
static std::mutex g_aux_mu;
static std::vector<AuxSet> g_aux_free;
static uint64_t g_aux_seq = 0;

// The pooled streams are destroyed at exit, before the HIP runtime's own teardown (an
// atexit handler registered after the runtime came up runs first): streams left to
// that teardown crashed the process at exit under rocprofv3.
static void release_aux_pool() {
  std::lock_guard<std::mutex> lk(g_aux_mu);
  for (AuxSet& a : g_aux_free) {
    (void)hipSetDevice(a.device);
    for (hipStream_t s : a.s) (void)hipStreamDestroy(s);
    (void)hipStreamDestroy(a.own);
    (void)hipStreamDestroy(a.cpy);
  }
  g_aux_free.clear();
}

static hipError_t take_aux(dm_ctx* c, int ncu) {
  {
    std::lock_guard<std::mutex> lk(g_aux_mu);
    size_t best = g_aux_free.size();
    for (size_t i = 0; i < g_aux_free.size(); ++i)
      if (g_aux_free[i].device == c->device && (best == g_aux_free.size() || g_aux_free[i].seq < g_aux_free[best].seq))
        best = i;
    if (best < g_aux_free.size()) {
      const AuxSet& a = g_aux_free[best];
      for (int k = 0; k < dm_ctx::kAux; ++k) c->aux[k] = a.s[k];
      c->own_stream = a.own;
      c->cpy = a.cpy;
      c->aux_own_queue = a.own_queue;
      c->aux_seq = a.seq;
      g_aux_free.erase(g_aux_free.begin() + (ptrdiff_t)best);
      return hipSuccess;
    }
    c->aux_seq = g_aux_seq++;
    static bool registered = false;
    if (!registered) registered = std::atexit(release_aux_pool) == 0;
  }
  const size_t mwords = (size_t)std::max(1, (ncu + 31) / 32);
  std::vector<uint32_t> mask(mwords, 0u);
  for (int b = 0; b < ncu; ++b) mask[(size_t)(b / 32)] |= 1u << (b % 32);
  c->aux_own_queue = true;
  // the creation order is measured (above)
  hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  for (int i = 0; i < dm_ctx::kAux && e == hipSuccess; ++i) {
    hipStream_t* slot = &c->aux[i];
    e = ncu > 0 ? hipExtStreamCreateWithCUMask(slot, (uint32_t)mwords, mask.data()) : hipErrorNotSupported;
    if (e != hipSuccess) {  // no CU masks here: a plain stream (correct, queue sharing as above)
      (void)hipGetLastError();
      c->aux_own_queue = false;
      e = hipStreamCreateWithFlags(slot, hipStreamNonBlocking);
    }
  }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->cpy, hipStreamNonBlocking);
  return e;
}

static void give_aux(dm_ctx* c) {
  if (!c->aux[0] || !c->own_stream || !c->cpy) return;
  (void)hipStreamSynchronize(c->own_stream);
  (void)hipStreamSynchronize(c->cpy);
  AuxSet a{c->device, c->aux_seq, {}, c->own_stream, c->cpy, c->aux_own_queue};
  c->own_stream = c->cpy = nullptr;
  for (int k = 0; k < dm_ctx::kAux; ++k) {
    (void)hipStreamSynchronize(c->aux[k]);
    a.s[k] = c->aux[k];
    c->aux[k] = nullptr;
  }
  std::lock_guard<std::mutex> lk(g_aux_mu);
  g_aux_free.push_back(a);
}

int dm_create(int device, dm_ctx** out) {
  if (!out) return DM_E_INVAL;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    g_last_error = std::string("no HIP device: ") + hipGetErrorString(e);
    return DM_E_HIP;
  }
  if (device < 0 || device >= n) {
    g_last_error = "device index out of range";
    return DM_E_RANGE;
  }
  e = hipSetDevice(device);
  if (e != hipSuccess) {
    g_last_error = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return DM_E_HIP;
  }
  dm_ctx* c = new dm_ctx();
  c->device = device;
  // Test hooks: each forces one of two product paths that the
  // library chooses between by itself, so that a test can compare the two on the same
  // ticks.  No other environment switch exists (round 5 retired the A/B probes).
  if (const char* df = getenv("DM_DECIDE_FAST")) c->decide_fast = atoi(df) != 0;
  if (const char* sc = getenv("DM_SPEC_CHAIN")) c->spec_chain = atoi(sc) != 0;
  if (const char* rl = getenv("DM_REDO_LIGHT")) c->redo_light = atoi(rl);
  if (const char* qc = getenv("DM_QUEUE_CALIB")) {  // 0: keep the creation-order queue assignment; 2: log
    if (atoi(qc) == 0) c->calib = 4;
    c->calib_log = atoi(qc) == 2;
  }
  if (const char* ds = getenv("DM_DENSE_SPLIT")) {
    const int v = (int)strtol(ds, nullptr, 0);
    c->dense_split = v == 1 ? 0xF : (v & 0xF);
  }
  e = hipSuccess;
  // The auxiliary streams are created with a full CU mask, which gives each its own
  // hardware queue.  Plain streams share the process's GPU_MAX_HW_QUEUES (4) queues
  // round robin with every other stream of the process (torch's included), so which
  // work classes ended up serialised behind one queue depended on how many streams
  // existed before: C2 tick 147-179 us by creation order, 147-151 us with the masks
  // (tools/host_cost.py, one process per run).  Static CU partitions (round 3-4 A/Bs:
  // 139-491 us against 136-140 us) and a high-priority chain stream (a queue shared
  // again) lost, and were retired in round 5.
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  // a quarter of headroom: the other classes' streams hold slots too, and run ahead
  // (DM_DEFER_JOIN)
  c->redo_cap = (int64_t)std::max(ncu, 1) * redo_blocks_per_cu() * 3 / 4;
  if (e == hipSuccess) e = take_aux(c, ncu);
  c->stream = c->own_stream;
  for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->ev_stage[i], hipEventDisableTiming);
  if (e == hipSuccess) e = xs_setup(c);
  for (auto& a : c->aset) {
    for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&a.ev_bat[i], hipEventDisableTiming);
    for (int i = 0; i < dm_ctx::kWChunks && e == hipSuccess; ++i)
      e = hipEventCreateWithFlags(&a.ev_wchunk[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&a.ev_done, hipEventDisableTiming);
  }
  for (int j = 0; j < dm_ctx::kParts; ++j)
    for (int i = 0; i < dm_ctx::kTickEv && e == hipSuccess; ++i) e = hipEventCreate(&c->tick_ev[j][i]);
  if (e != hipSuccess) {
    g_last_error = std::string("stream/event setup: ") + hipGetErrorString(e);
    dm_destroy(c);
    return DM_E_HIP;
  }
  *out = c;
  return DM_OK;
}

struct RcclApi;
static const RcclApi* rccl_api();
static void rccl_destroy(const RcclApi* r, ncclComm_t comm);

static void calib_free(dm_ctx* c);

void dm_destroy(dm_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->nccl_comm) {
    rccl_destroy(rccl_api(), c->nccl_comm);
    c->nccl_comm = nullptr;
  }
  // deferred tick work (DM_DEFER_JOIN) and update copies may still run on the
  // auxiliary streams: drain every stream before any buffer is freed
  for (int i = 0; i < dm_ctx::kAux; ++i)
    if (c->aux[i]) (void)hipStreamSynchronize(c->aux[i]);
  if (c->cpy) (void)hipStreamSynchronize(c->cpy);
  (void)hipStreamSynchronize(c->stream);
  c->collect_profile();
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  calib_free(c);
  c->free_all();
  give_aux(c);  // kept for the next context on this device (take_aux)
  for (int i = 0; i < dm_ctx::kAux; ++i)  // (a set not returned whole)
    if (c->aux[i]) (void)hipStreamDestroy(c->aux[i]);
  if (c->cpy) {
    (void)hipStreamSynchronize(c->cpy);
    (void)hipStreamDestroy(c->cpy);
  }
  for (int i = 0; i < dm_ctx::XS_N; ++i)
    if (c->xs_ev[i]) (void)hipEventDestroy(c->xs_ev[i]);
  for (auto ev : c->ev_stage)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& a : c->aset) a.destroy_events();
  for (auto& row : c->tick_ev)
    for (auto ev : row)
      if (ev) (void)hipEventDestroy(ev);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char* dm_last_error(dm_ctx* c) { return c ? c->err.c_str() : g_last_error.c_str(); }

int dm_set_stream(dm_ctx* c, void* s) {
  DM_ENTER(c);
  DM_HIP(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  // the template slots' lazy signals on the old stream are complete now, and that
  // stream may not outlive this call: never record on it again
  for (int i = 0; i < dm_ctx::kTplSlots; ++i)
    for (dm_ctx::XsTok* t : {&c->tpl_ready[i], &c->tpl_free[i]})
      if (!t->rec && t->s == c->stream) t->s = nullptr;
  c->stream = s ? (hipStream_t)s : c->own_stream;
  c->main_dirty = true;
  return DM_OK;
}

void* dm_get_stream(dm_ctx* c) { return c ? (void*)c->stream : nullptr; }

int dm_join(dm_ctx* c) {
  DM_ENTER(c);
  return DM_OK;
}

int dm_stream_wait(dm_ctx* c, void* s) {
  DM_ENTER(c);
  if (!s) return c->fail(DM_E_INVAL, "null stream");
  DM_HIP(c, c->xs_order(dm_ctx::XS_EXT, c->stream, (hipStream_t)s), "stream order");
  return DM_OK;
}

int dm_sync(dm_ctx* c) {
  DM_ENTER(c);
  const int rc = c->synced("hipStreamSynchronize");
  c->collect_profile();
  return rc;
}

// Asynchronous store batches still in flight finish before the store or its
// configuration is replaced (their outcome is dropped with the store they updated).
static void async_drain(dm_ctx* c) {
  for (int i = 1; i <= dm_ctx::kAsyncSets; ++i)
    if (c->aset[i].pending) {
      (void)hipEventSynchronize(c->aset[i].ev_done);
      c->aset[i].pending = false;
    }
}

int dm_store_load(dm_ctx* c, const dm_snapshot* s) {
  DM_ENTER(c);
  async_drain(c);
  if (!s || s->n_resources < 0 || s->n_leases < 0 || !s->seg_off) return c->fail(DM_E_INVAL, "bad snapshot");
  const int64_t R = s->n_resources, N = s->n_leases;
  if (R > INT32_MAX - 1) return c->fail(DM_E_INVAL, "too many resources for one context (max 2^31-2)");
  if (N > 0 && (!s->wants || !s->has || !s->subclients || !s->expiry_ns))
    return c->fail(DM_E_INVAL, "snapshot columns missing");
  if (s->seg_off[0] != 0 || s->seg_off[R] != N) return c->fail(DM_E_INVAL, "seg_off must run from 0 to n_leases");
  for (int64_t r = 0; r < R; ++r)
    if (s->seg_off[r + 1] < s->seg_off[r]) return c->fail(DM_E_INVAL, "seg_off must be non-decreasing");
  for (int64_t i = 0; i < N; ++i)
    if (s->subclients[i] < 0 || s->subclients[i] > kSubMax)
      return c->fail(DM_E_INVAL, "subclients must be in [0, 2^31-2]");
  const bool have_agg = s->agg_count && s->agg_sum_has && s->agg_sum_wants;
  if ((s->agg_count || s->agg_sum_has || s->agg_sum_wants) && !have_agg)
    return c->fail(DM_E_INVAL, "give all three running sums or none");
  DM_HIP(c, hipStreamSynchronize(c->stream), "sync");
  c->R = R;
  c->N = N;
  c->h_seg_off.assign(s->seg_off, s->seg_off + R + 1);
  c->seg_uniform = 0;  // every resource the same number of rows (a hierarchy root store: G)
  if (R > 0) {
    const int64_t g = s->seg_off[1] - s->seg_off[0];
    bool same = g > 0 && s->seg_off[0] == 0;
    for (int64_t r = 1; r < R && same; ++r) same = s->seg_off[r + 1] - s->seg_off[r] == g;
    c->seg_uniform = same ? g : 0;
  }
  hipStream_t st = c->stream;
  DM_HIP(c, upload(c->seg_off, s->seg_off, (size_t)R + 1, st), "upload seg_off");
  {  // RowIndex: resource of the first row of every 2^kRowBlkShift-row block
    const int64_t nb = (N >> kRowBlkShift) + 2;
    std::vector<int32_t> blk((size_t)nb, 0);
    int64_t sg = 0;
    for (int64_t b = 0; b < nb && R > 0; ++b) {
      const int64_t row = std::min<int64_t>(b << kRowBlkShift, std::max<int64_t>(N - 1, 0));
      while (sg + 1 < R && s->seg_off[sg + 1] <= row) ++sg;
      blk[(size_t)b] = (int32_t)sg;
    }
    DM_HIP(c, upload(c->blk_seg, blk.data(), blk.size(), st), "upload row index");
    DM_HIP(c, hipStreamSynchronize(st), "upload row index");  // blk leaves scope
  }
  DM_HIP(c, upload(c->wants, s->wants, (size_t)N, st), "upload wants");
  DM_HIP(c, upload(c->has, s->has, (size_t)N, st), "upload has");
  {
    std::vector<int32_t> sub32((size_t)N);
    // every loaded row keeps its own expiry (explicit, dm_device.h); a writeback tick
    // turns the live ones into followers of their resource's expiry
    for (int64_t i = 0; i < N; ++i) sub32[i] = (int32_t)((uint32_t)s->subclients[i] | kSubExplicit);
    DM_HIP(c, upload(c->sub, sub32.data(), (size_t)N, st), "upload subclients");
    DM_HIP(c, hipStreamSynchronize(st), "upload subclients");  // sub32 leaves scope
  }
  DM_HIP(c, upload(c->expiry, s->expiry_ns, (size_t)N, st), "upload expiry");
  std::vector<int64_t> cnt;
  std::vector<double> sh, sw;
  const int64_t* ac = s->agg_count;
  const double* ah = s->agg_sum_has;
  const double* aw = s->agg_sum_wants;
  if (!have_agg) {  // one Assign per row, in row order (store.go:156-158)
    cnt.assign(R, 0);
    sh.assign(R, 0.0);
    sw.assign(R, 0.0);
    for (int64_t r = 0; r < R; ++r)
      for (int64_t i = s->seg_off[r]; i < s->seg_off[r + 1]; ++i) {
        sh[r] += s->has[i] - 0.0;
        sw[r] += s->wants[i] - 0.0;
        cnt[r] += s->subclients[i];
      }
    ac = cnt.data();
    ah = sh.data();
    aw = sw.data();
  }
  std::vector<ResAgg> agg(R);
  for (int64_t r = 0; r < R; ++r) agg[r] = ResAgg{ac[r], ah[r], aw[r], 0};
  DM_HIP(c, upload(c->agg, agg.data(), (size_t)R, st), "upload running sums");
  const std::vector<uint8_t> expl((size_t)std::max<int64_t>(R, 1), 1);  // loaded rows carry explicit expiries
  DM_HIP(c, upload(c->expl, expl.data(), expl.size(), st), "upload explicit flags");
  DM_HIP(c, c->rmask.ensure((size_t)(N / 2 + 64)), "alloc released-row masks");  // zeroed by upload_plan
  build_plan(c);
  int rc = upload_plan(c);
  if (rc) return rc;
  c->maybe_general = scan_maybe_general(s->seg_off, R, s->subclients, s->wants, s->expiry_ns);
  // released rows never take part in a tick, so they do not count against this
  c->all_sub_one = true;
  for (int64_t i = 0; i < N && c->all_sub_one; ++i)
    c->all_sub_one = s->subclients[i] == 1 || s->expiry_ns[i] == DM_RELEASED;
  DM_HIP(c, hipStreamSynchronize(st), "store load");
  c->store_loaded = true;
  c->store_lost = false;  // upload_plan cleared the device's failure words
  c->expl_rows = true;
  c->rows_changed();
  c->have_result = false;
  c->hints_set = false;
  if (c->cfg_loaded && (int64_t)c->h_refresh_s.size() != R) c->cfg_loaded = false;
  return DM_OK;
}

int dm_config_load(dm_ctx* c, int64_t R, const dm_resource_cfg* cfg) {
  DM_ENTER(c);
  async_drain(c);  // (an in-flight batch's arrivals take the lease lengths they were sent under)
  c->rows_changed();
  if (!cfg || R < 0 || !cfg->kind || !cfg->capacity || !cfg->lease_length_s || !cfg->refresh_interval_s ||
      !cfg->learning_end_ns || !cfg->parent_expiry_ns || !cfg->safe_capacity)
    return c->fail(DM_E_INVAL, "bad config");
  for (int64_t r = 0; r < R; ++r) {
    if (cfg->lease_length_s[r] < 0 || cfg->refresh_interval_s[r] < 0)
      return c->fail(DM_E_INVAL, "lease_length and refresh_interval must be >= 0 (server.go:384-434)");
    if (cfg->refresh_interval_s[r] > INT32_MAX || cfg->lease_length_s[r] > INT32_MAX)
      return c->fail(DM_E_INVAL, "refresh_interval and lease_length must be < 2^31 s");
  }
  for (int64_t r = 0; r < R; ++r)
    if (cfg->kind[r] < DM_NO_ALGORITHM || cfg->kind[r] > DM_FAIR_SHARE) {
      char buf[96];
      snprintf(buf, sizeof buf, "unknown algorithm kind %d for resource %lld", cfg->kind[r], (long long)r);
      return c->fail(DM_E_KIND, buf);
    }
  DM_HIP(c, hipStreamSynchronize(c->stream), "sync");
  hipStream_t st = c->stream;
  std::vector<ResCfg> rc(R);
  std::vector<ResCold> rcold(R);
  for (int64_t r = 0; r < R; ++r) {
    rc[r] = ResCfg{cfg->capacity[r], cfg->learning_end_ns[r], cfg->parent_expiry_ns[r],
                   (int32_t)cfg->lease_length_s[r], cfg->kind[r]};
    rcold[r] = ResCold{cfg->safe_capacity[r], (int32_t)cfg->refresh_interval_s[r], 0};
  }
  c->tpl_pending.clear();  // staged exchanges were computed for the old configuration
  DM_HIP(c, upload(c->cfg, rc.data(), (size_t)R, st), "upload config");
  DM_HIP(c, upload(c->cold, rcold.data(), (size_t)R, st), "upload config");
  c->h_refresh_s.assign(cfg->refresh_interval_s, cfg->refresh_interval_s + R);
  c->h_kind.assign(cfg->kind, cfg->kind + R);
  if (c->store_loaded && R == c->R) {  // bin 4's shape by the new kinds
    if (int rc2 = update_bin4_shape(c, st)) return rc2;
  }
  DM_HIP(c, hipStreamSynchronize(st), "config load");
  c->cfg_loaded = true;
  return DM_OK;
}

static int ready(dm_ctx* c) {
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (int rc = c->check_device()) return rc;
  if (!c->cfg_loaded || (int64_t)c->h_refresh_s.size() != c->R)
    return c->fail(DM_E_STATE, "no configuration loaded for the store's resources");
  return DM_OK;
}

// Pipelined hierarchy (dm_hier_pipeline): before a leaf tick, take the templates of
// the exchanges enqueued before the previous tick (stream-ordered after their root
// kernels); the slot they replace becomes free once the ticks that read it are done.
static int commit_templates(dm_ctx* c) {
  int take = -1;
  size_t n = 0;
  while (n < c->tpl_pending.size() && c->tpl_pending[n].tag + (c->tpl_lag - 1) < c->ticks_issued)
    take = c->tpl_pending[n++].slot;
  for (size_t i = 0; i + 1 < n; ++i) c->tpl_free_slots.push_back(c->tpl_pending[i].slot);  // superseded
  c->tpl_pending.erase(c->tpl_pending.begin(), c->tpl_pending.begin() + (ptrdiff_t)n);
  if (take < 0) return DM_OK;
  const dm_ctx::XsTok& rt = c->tpl_ready[take];
  const bool host_wait = rt.rec && rt.s && rt.s != c->stream;
  // deferred class work also read the old templates: joined, unless the last tick's
  // events cover it (the slot's reuse then waits on them, below)
  const bool keep = host_wait && c->tick_covers();
  if (!keep) DM_HIP(c, c->join_aux(), "join");
  if (host_wait) {
    // poll: the wake-up of a blocking wait comes too late for the next launch to be
    // queued in time.  Bounded by time (the exchange may wait on a slower rank's
    // all-gather): after 50 us of polling, a blocking wait frees the core.
    hipError_t q = hipEventQuery(c->xs_ev[rt.w]);
    if (q == hipErrorNotReady) {
      timespec t0{}, t1{};
      clock_gettime(CLOCK_MONOTONIC, &t0);
      do {
        q = hipEventQuery(c->xs_ev[rt.w]);
        clock_gettime(CLOCK_MONOTONIC, &t1);
      } while (q == hipErrorNotReady &&
               (t1.tv_sec - t0.tv_sec) * 1000000000LL + (t1.tv_nsec - t0.tv_nsec) < 50000);
    }
    if (q == hipErrorNotReady) q = hipEventSynchronize(c->xs_ev[rt.w]);
    if (q != hipSuccess) return c->hip_fail(q, "staged templates");
  } else {
    DM_HIP(c, c->xs_wait(rt, c->stream), "staged templates");
  }
  if (!keep) c->main_dirty = true;  // the class streams fork after the wait
  std::swap(c->cfg, c->tpl_cfg[take]);
  std::swap(c->cold, c->tpl_cold[take]);
  // the old templates (now in slot `take`) are free after the ticks already enqueued
  // the next exchange into it waits for the ticks enqueued so far: on the last tick's
  // events (tick_ev, every stream part's) when its last kernels complete them, else on
  // a (lazy) event
  c->tpl_free_seq[take] = c->tick_flagged ? c->tick_seq : 0;
  c->xs_signal_lazy(dm_ctx::XS_FREE0 + take, c->stream, &c->tpl_free[take]);
  c->tpl_free_rec[take] = true;
  c->tpl_free_slots.push_back(take);
  return DM_OK;
}

// One forked writeback tick's part in the queue calibration (dm_ctx::calib), called
// before the tick forks.  Window boundaries join every class stream into the context
// stream (so the next window's assignment starts after the last one's work: a class's
// consecutive ticks on two streams are then still ordered) and record an event there.
static hipError_t calib_apply(dm_ctx* c, const std::array<int, dm_ctx::kAux>& pm) {
  hipError_t e = c->join_aux();
  if (e != hipSuccess) return e;
  for (int i = 0; i < dm_ctx::kAux; ++i) {
    c->perm[i] = pm[(size_t)i];
    c->aux[i] = c->aux_phys[pm[(size_t)i]];
  }
  c->main_dirty = true;  // the next tick forks: every class stream waits for the context stream
  return hipSuccess;
}

static hipError_t calib_mark(dm_ctx* c, bool end) {
  if (end) {
    hipEvent_t ev;
    hipError_t e = c->join_aux();
    if (e == hipSuccess) e = hipEventCreate(&ev);
    if (e == hipSuccess) e = hipEventRecord(ev, c->stream);
    if (e != hipSuccess) return e;
    c->calib_ev.back().second = ev;
    c->main_dirty = true;
    return hipSuccess;
  }
  hipEvent_t ev;
  hipError_t e = hipEventCreate(&ev);
  if (e == hipSuccess) e = hipEventRecord(ev, c->stream);
  if (e != hipSuccess) return e;
  c->calib_ev.push_back({ev, nullptr});
  c->calib_of_ev.push_back(c->calib_k);
  return hipSuccess;
}

static void calib_free(dm_ctx* c) {
  for (auto& pr : c->calib_ev) {
    if (pr.first) (void)hipEventDestroy(pr.first);
    if (pr.second) (void)hipEventDestroy(pr.second);
  }
  c->calib_ev.clear();
  c->calib_of_ev.clear();
}

static hipError_t calib_step(dm_ctx* c) {
  if (c->calib == 4) return hipSuccess;
  if (c->calib == 0) {
    if (!c->aux_own_queue) {  // shared queues: the assignment does not choose hardware queues
      c->calib = 4;
      return hipSuccess;
    }
    if (++c->calib_skip < dm_ctx::kCalibSkip) return hipSuccess;
    for (int i = 0; i < dm_ctx::kAux; ++i) c->aux_phys[i] = c->aux[i];
    std::array<int, dm_ctx::kAux> pm{0, 1, 2, 3};
    c->calib_cand.clear();
    do c->calib_cand.push_back(pm);
    while (std::next_permutation(pm.begin(), pm.end()));
    c->calib = 1;
    c->calib_round = 1;
    c->calib_k = 0;
    c->calib_t = 1;  // this tick is the window's first
    hipError_t e = calib_apply(c, c->calib_cand[0]);
    return e == hipSuccess ? calib_mark(c, false) : e;
  }
  if (c->calib == 1 || c->calib == 2) {
    const int win = c->calib == 1 ? dm_ctx::kCalibWin : dm_ctx::kCalibWin2;
    if (++c->calib_t <= win) return hipSuccess;
    hipError_t e = calib_mark(c, true);
    if (e != hipSuccess) return e;
    c->calib_t = 1;
    const int ncand = (int)c->calib_cand.size();
    if (++c->calib_k < ncand) {
      e = calib_apply(c, c->calib_cand[(size_t)c->calib_k]);
      return e == hipSuccess ? calib_mark(c, false) : e;
    }
    c->calib = 3;  // wait for the windows' events (polled by later ticks)
    return hipSuccess;
  }
  // calib == 3: the last window's end event done?  then pick
  const hipError_t q = hipEventQuery(c->calib_ev.back().second);
  if (q == hipErrorNotReady) return hipSuccess;
  if (q != hipSuccess) return q;
  std::vector<std::pair<float, size_t>> t;
  for (size_t w = 0; w < c->calib_ev.size(); ++w) {
    float ms = 0.0f;
    hipError_t e = hipEventElapsedTime(&ms, c->calib_ev[w].first, c->calib_ev[w].second);
    if (e != hipSuccess) return e;
    t.push_back({ms, w});
  }
  if (c->calib_log) {  // test hook (DM_QUEUE_CALIB=2): every window's assignment and time per tick
    const int win = c->calib_round == 1 ? dm_ctx::kCalibWin : dm_ctx::kCalibWin2;
    for (const auto& pr : t) {
      const auto& pm = c->calib_cand[(size_t)c->calib_of_ev[pr.second]];
      fprintf(stderr, "[dm queue calibration] round %d perm %d%d%d%d %.2f us/tick\n", win == dm_ctx::kCalibWin ? 1 : 2,
              pm[0], pm[1], pm[2], pm[3], 1000.0 * pr.first / win);
    }
  }
  std::sort(t.begin(), t.end());
  if (c->calib == 3 && c->calib_round == 1) {  // round 2: the best of round 1 over longer windows
    // the best kCalibFinal of round 1, and the creation-order assignment (the measured
    // default) so that the choice is never worse than not calibrating
    std::vector<std::array<int, dm_ctx::kAux>> fin;
    const std::array<int, dm_ctx::kAux> ident{0, 1, 2, 3};
    for (int i = 0; i < dm_ctx::kCalibFinal; ++i) fin.push_back(c->calib_cand[(size_t)c->calib_of_ev[t[(size_t)i].second]]);
    if (std::find(fin.begin(), fin.end(), ident) == fin.end()) fin.push_back(ident);
    calib_free(c);
    c->calib_cand.clear();
    for (int r = 0; r < dm_ctx::kCalibRep2; ++r)  // interleaved: fin[0], fin[1], ..., fin[0], ...
      c->calib_cand.insert(c->calib_cand.end(), fin.begin(), fin.end());
    c->calib = 2;
    c->calib_round = 2;
    c->calib_k = 0;
    c->calib_t = 1;
    hipError_t e = calib_apply(c, c->calib_cand[0]);
    return e == hipSuccess ? calib_mark(c, false) : e;
  }
  // round 2: each candidate's windows summed
  std::vector<std::pair<std::array<int, dm_ctx::kAux>, float>> sum;
  for (const auto& pr : t) {
    const auto& pm = c->calib_cand[(size_t)c->calib_of_ev[pr.second]];
    auto it = std::find_if(sum.begin(), sum.end(), [&](const auto& x) { return x.first == pm; });
    if (it == sum.end()) sum.push_back({pm, pr.first});
    else it->second += pr.first;
  }
  const auto best = std::min_element(sum.begin(), sum.end(), [](const auto& a, const auto& b) {
                      return a.second < b.second;
                    })->first;
  calib_free(c);
  c->calib = 4;
  c->calib_best = best[0] + 4 * best[1] + 16 * best[2] + 64 * best[3];
  return calib_apply(c, best);
}

int dm_apportion(dm_ctx* c, int64_t now_ns, uint32_t flags) {
  DM_CHECK_CTX(c);
  int rc = ready(c);
  if (rc) return rc;
  if (c->tpl_pipe && (rc = commit_templates(c))) return rc;
  c->ticks_issued += 1;
  c->tick_seq += 1;
  c->tick_flagged = false;
  const bool wb = flags & DM_WRITEBACK;
  DevParams p{};
  p.seg_off = c->seg_off.p;
  p.wants = c->wants.p;
  p.has = c->has.p;
  p.sub = c->sub.p;
  p.expiry = c->expiry.p;
  p.cfg = c->cfg.p;
  p.agg = c->agg.p;
  p.expl = c->expl.p;
  p.rmask = c->rmask.p;
  // Every tick writes every row's lease (released rows included).  On a store
  // beyond the Infinity Cache a writeback tick writes its gets/expiry into the
  // alternate pair of columns and the pairs swap afterwards: separate output
  // columns stream faster than in-place read-then-write of the same lines (C3,
  // 100M rows: 815 -> 760 us per tick, tools/ab.py).  A
  // cache-resident store (C1, 440 MB) keeps in-place writes, which the cache
  // serves better (72 vs 76 us).
  if ((flags & DM_WB_INPLACE) && (flags & DM_WB_ALTERNATE))
    return c->fail(DM_E_INVAL, "DM_WB_INPLACE and DM_WB_ALTERNATE are exclusive");
  // The speculative large chain (below) writes its gets before they are verified, so a
  // tick that may take it writes the alternate column whatever the store's size.
  const bool spec_eligible = c->spec_chain && wb && !(flags & DM_AGG_RECOMPUTE) && !c->expl_rows &&
                             !((c->maybe_general || c->async_may_general()) && c->n_nonsmall > 0) &&
                             !c->h_chunks.empty();
  const bool pingpong = wb && !(flags & DM_WB_INPLACE) &&
                        ((flags & DM_WB_ALTERNATE) || c->N * 48 > kStreamBytes || spec_eligible);
  // A writeback tick writes no per-lease expiry: the leases it grants follow their
  // resource's expiry (dm_device.h), so only gets (and rare subclients words) move.
  if (!wb) {
    DM_HIP(c, c->out_gets.ensure((size_t)std::max<int64_t>(c->N, 1)), "alloc out_gets");
    DM_HIP(c, c->out_expiry.ensure((size_t)std::max<int64_t>(c->N, 1)), "alloc out_expiry");
    p.out_gets = c->out_gets.p;
    p.out_expiry = c->out_expiry.p;
  } else if (pingpong) {
    DM_HIP(c, c->out_gets.ensure((size_t)std::max<int64_t>(c->N, 1)), "alloc out_gets");
    p.out_gets = c->out_gets.p;
    p.out_expiry = nullptr;
  } else {
    p.out_gets = c->has.p;
    p.out_expiry = nullptr;
  }
  p.writeback = wb ? 1 : 0;
  if (wb) {
    p.out_wants = c->wants.p;
    p.out_sub = c->sub.p;
    p.res = c->agg.p;
  } else {
    DM_HIP(c, c->res.ensure((size_t)std::max<int64_t>(c->R, 1)), "alloc res");
    p.out_wants = nullptr;
    p.out_sub = nullptr;
    p.res = c->res.p;
  }
  p.now = now_ns;
  p.recompute = (flags & DM_AGG_RECOMPUTE) ? 1 : 0;
  const bool live_ok = c->chain_live_ok;
  c->chain_live_ok = false;
  bool chain_live = false;  // this tick ran the (non-heterogeneous) chain
  if (wb && !c->pub_ring.empty()) {
    const int64_t n = (int64_t)c->pub_ring.size();
    p.pub = c->pub_ring[(size_t)(c->pub_k % n)];
    p.pub_clear = c->pub_ring[(size_t)((c->pub_k + 1) % n)];
    p.pub_word = -1;  // (a split bin's parts set their own)
    p.pub_first = 0;
    c->pub_k += 1;
  }

  Partials P{c->pa_cnt.p, c->pa_has.p, c->pa_wants.p, c->pa_cnt_all.p, c->pa_has_all.p, c->pa_wants_all.p,
             c->pa_smin.p, c->pa_smax.p, c->pa_nan.p,
             c->pb_x.p,   c->pb_y.p,   c->pb_w.p,     c->pc_ee.p,   c->pc_sgt.p,  c->pd_delta.p,
             c->pa_live.p, c->p_tot.p, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipStream_t st = c->stream;
  auto timed = [&](int cls, hipStream_t s, auto&& fn) -> hipError_t { return c->timed(cls, s, fn); };
  const int nch = (int)c->h_chunks.size();
  int32_t* gl = c->glist.p;
  int32_t* gc = c->gcount.p;
  // (an asynchronous store batch still in flight may bring NaN wants or other subclient
  // counts: the tick is ready for k_general until the batch is retired)
  const bool general = (c->maybe_general || c->async_may_general()) && c->n_nonsmall > 0;
  if (general) {  // only non-small resources are ever appended to the worklist
    DM_HIP(c, hipMemsetAsync(gc, 0, sizeof(int32_t), st), "worklist reset");
    c->main_dirty = true;
  }
  // Independent work classes: large resources (a 5-kernel chain), big groups,
  // small groups + packed.  With more than one class present they run on the
  // auxiliary streams concurrently, forked from and joined back to the main stream.
  unsigned used = 0;  // auxiliary streams with work this tick
  for (int b = 0; b < kNumBins; ++b)
    if (!c->h_bins[b].empty()) {
      used |= 1u << c->class_stream[b];
      if (c->bin_parts[b] > 1) used |= 1u << c->part_stream(b, 1);
    }
  if (!c->h_tiles.empty()) used |= 1u << c->class_stream[kNumBins];
  if (nch > 0) used |= 1u << c->class_stream[kNumBins + 1];
  const bool fork = __builtin_popcount(used) > 1;
  int nonempty_bins = 0;
  for (int b = 0; b < kNumBins; ++b) nonempty_bins += c->h_bins[b].empty() ? 0 : 1;
  // one work class (on the context stream, or in stream parts): its split bin's last
  // kernel completes the tick's event (only check_dense's hint count may follow it)
  bool parts_only = false;
  for (int b = 0; b < kNumBins; ++b) parts_only |= !c->h_bins[b].empty() && c->bin_parts[b] > 1;
  const bool one_class = (!fork || parts_only) && nch == 0 && c->h_tiles.empty() && !general && nonempty_bins == 1;
  if (fork && wb && c->tick_signal_wanted == false) DM_HIP(c, calib_step(c), "queue calibration");
  auto cls_stream = [&](int cls) { return fork ? c->aux[c->class_stream[cls]] : st; };
  hipStream_t s_large = cls_stream(kNumBins + 1), s_small = cls_stream(kNumBins);
  if (!fork) {  // everything on the context stream, after any deferred class work
    DM_HIP(c, c->join_aux(), "join");
    c->main_dirty = true;
  } else if (c->main_dirty) {  // class streams wait for what the context stream holds
    dm_ctx::XsTok fk;
    DM_HIP(c, c->xs_signal(dm_ctx::XS_FORK, st, &fk), "fork");
    for (int i = 0; i < dm_ctx::kAux; ++i) DM_HIP(c, c->xs_wait(fk, c->aux[i]), "fork");
    c->main_dirty = false;
  }
  if (fork) c->aux_unjoined |= used;
  {
    const int nls = (int)c->h_large.size();
    // heterogeneous-subclient FairShare is decided on the chain when the store may
    // hold it (k_large_t, k_large_c_het, k_large_e, k_large_map_het)
    const bool het = general && nch > 0;
    if (het) {
      const size_t nc = (size_t)nch, nl = (size_t)std::max(nls, 1);
      if (c->ph_set_ready < nl || c->ph_set.n < nl * 2 * kHetMaxS) {
        DM_HIP(c, c->ph_set.ensure(nl * 2 * kHetMaxS), "heterogeneous partials");
        DM_HIP(c, c->ph_n.ensure(nl), "heterogeneous partials");
        DM_HIP(c, hipMemsetAsync(c->ph_set.p, 0xFF, nl * 2 * kHetMaxS * sizeof(uint32_t), s_large), "heterogeneous sets");
        DM_HIP(c, hipMemsetAsync(c->ph_n.p, 0, nl * sizeof(int32_t), s_large), "heterogeneous sets");
        c->ph_set_ready = nl;
      }
      DM_HIP(c, c->ph_het.ensure(nl * sizeof(HetRes)), "heterogeneous partials");
      DM_HIP(c, c->ph_bkw.ensure(nc * kHetBuckets), "heterogeneous partials");
      DM_HIP(c, c->ph_bks.ensure(nc * kHetBuckets), "heterogeneous partials");
      DM_HIP(c, c->ph_bkc.ensure(nc * kHetBuckets), "heterogeneous partials");
      P.s_set = c->ph_set.p;
      P.s_n = c->ph_n.p;
      P.het = c->ph_het.p;
      P.bk_w = c->ph_bkw.p;
      P.bk_s = c->ph_bks.p;
      P.bk_c = c->ph_bkc.p;
    }
    P.b_first = (!het && !p.recompute && !c->expl_rows) ? 1 : 0;
    P.s_live = (!het && live_ok && !c->expl_rows) ? 1 : 0;
    P.uni = c->p_uni.p;
    // A, B, [T], C, [C_het, E], map, [map_het], fin
    static constexpr int kSeq[9] = {0, 1, 5, 2, 6, 7, 3, 8, 4};
    static constexpr int kCls[9] = {KC_LARGE_A, KC_LARGE_B,   KC_LARGE_T,  KC_LARGE_C,  KC_LARGE_CH,
                                    KC_LARGE_E, KC_LARGE_MAP, KC_LARGE_MH, KC_LARGE_FIN};
    // the steady state: one speculative launch, verified per resource, and a redo launch
    // that only the resources whose totals moved use (the store's rows must not be
    // overwritten by the speculative gets: alternate output columns)
    const bool spec = c->spec_chain && !het && P.b_first && wb && p.out_gets != p.has && nch > 0;
    if (spec) {
      const SpecArgs S{c->p_spec.p, c->spec_seq, c->d_serr, c->p_spec_ring.p, (int)(c->spec_seq & 1), nch,
                       reinterpret_cast<uint32_t*>(c->d_serr + 1), c->p_team.p, c->nslots};
      c->spec_seq += 1;
      const bool light = c->redo_light == 2 || (c->redo_light == 1 && c->redo_epoch == c->row_epoch &&
                                                __atomic_exchange_n(c->h_serr + 1, 0, __ATOMIC_RELAXED) == 0);
      c->redo_epoch = c->row_epoch;
      const int redo_phase = light ? 2 : 1;
      const int redo_grid = light ? c->team_grid_light : c->team_grid_full;
      for (int ph = 0; ph < 2; ++ph)
        DM_HIP(c, timed(ph == 0 ? KC_LARGE_SPEC : KC_LARGE_REDO, s_large,
                        [&] {
                          return launch_large_spec(ph == 0 ? 0 : redo_phase, p, c->chunks.p, nch, c->large.p, P, S,
                                                   redo_grid, gl, gc, s_large);
                        }),
               "large-resource kernels");
    }
    for (int i = 0; i < 9 && nch > 0 && !spec; ++i) {
      const int ph = kSeq[i];
      if (ph >= 5 && !het) continue;
      if (ph == 4 && !het) continue;  // the map's last-arriving chunks did fin's work
      DM_HIP(c, timed(kCls[i], s_large,
                      [&] { return launch_large(ph, p, c->chunks.p, nch, c->large.p, nls, P, gl, gc, s_large); }),
             "large-resource kernels");
    }
    chain_live = nch > 0 && !het;
  }
  // the workgroup bins split by the dense hint after a writeback tick (hints set)
  const bool split_dense = c->hints_set;
  // the sub-wave bins (8x2, 16x2, 16x4, 32x4, 64x4) in one launch on bin 0's stream
  {
    SubBins sb{};
    int nonempty = 0;
    for (int k = 0; k < kSubShapes; ++k) {  // each sub-wave bin's items by shape (build_plan)
      const int b = kSubShapeBin[k], n = (int)c->h_shape_n[k];
      const int per = 256 / kSubShapeG[k];
      sb.items[k] = c->bins[b].p + c->h_shape_lo[k];
      sb.n[k] = n;
      sb.blocks[k] = (n + per - 1) / per;
      nonempty += n > 0;
    }
    if (nonempty > 0) {
      hipStream_t s = cls_stream(0);
      DM_HIP(c, timed(KC_SUBS, s, [&] { return launch_subs(p, sb, gl, gc, s); }), "sub-wave kernel");
    }
  }
  for (int b = kNumBins - 1; b >= 0; --b) {
    if (c->h_bins[b].empty()) continue;
    if (b == 7 || b == 8 || b <= 2) continue;  // k_subs
    const int lb = (b == 6 && c->bin6_wide)   ? kBin6Wide
                   : (b == 4 && c->bin4_wave) ? kBin4Wave
                                              : b;  // the launchers' bin (shape)
    const int nparts = c->bin_parts[b];
    if (one_class && c->tick_signal_wanted) {
      c->tick_flagged = true;
      c->tick_nev[c->tick_seq % dm_ctx::kTickEv] = nparts;
      c->tick_part_mask = 0;
    }
    for (int j = 0; j < nparts; ++j) {
      const int64_t lo = c->part_lo[b][j];
      const int n = (int)(c->part_lo[b][j + 1] - lo);
      if (n == 0) continue;
      WorkItem* items = c->bins[b].p + lo;
      hipStream_t s = j == 0 ? cls_stream(b) : c->aux[c->part_stream(b, j)];
      DevParams pj = p;
      if (nparts > 1 && p.pub) {  // the part's own flags word (DevParams::pub_word)
        pj.pub_word = j;
        pj.pub_first = c->h_bins[b][(size_t)lo].seg;
      }
      // the tick's last kernel of this part (the dense kernel, or the rest kernel after
      // it) completes the part's tick event when another queue waits for the tick
      hipEvent_t done = nullptr;
      if (one_class && c->tick_signal_wanted) {
        done = c->tick_ev[j][c->tick_seq % dm_ctx::kTickEv];
        c->tick_part_mask |= fork ? 1u << (j == 0 ? c->class_stream[b] : c->part_stream(b, j)) : 0u;
      }
      const int i = (b - 3) * dm_ctx::kParts + j;  // split slot (bins 3-6)
      if (b >= 3 && b < 3 + dm_ctx::kSplitBins && ((c->dense_split >> (b - 3)) & 1) && split_dense) {
        // only a writeback tick sets hints, so the split form follows one
        const int par = c->dq_par[i];
        const int64_t queued = __atomic_load_n(c->h_dq + i, __ATOMIC_RELAXED);
        const bool good = 4 * queued <= n;
        if (good) c->dq_wait[i] = 64;
        if (good || ++c->dq_skip[i] >= c->dq_wait[i]) {
          if (!good) c->dq_wait[i] = std::min(2 * c->dq_wait[i], 4096);
          c->dq_skip[i] = 0;
          // Every item verified dense in this row epoch: nothing can be queued, so the
          // dense kernel is the part's only launch (the guard catches the impossible).
          const uint64_t* rec = c->h_rec + 2 * i;
          const bool skip = __atomic_load_n(rec + 1, __ATOMIC_ACQUIRE) == c->row_epoch &&
                            __atomic_load_n(rec, __ATOMIC_RELAXED) == 0;
          DM_HIP(c, timed(KC_DENSE3 + (b - 3), s, [&] {
                   return launch_bin_dense(lb, pj, items, n, c->dq_list[i].p, c->dq_cnt[i].p, par, gl, gc,
                                           skip ? c->d_guard + i : nullptr, skip ? done : nullptr, s);
                 }),
                 "group kernel (dense split)");
          if (!skip) {
            // the rest kernel strides over whatever the dense kernel queues; its grid is
            // only sized from the last split tick's queue (a hint: correctness never
            // depends on it): an empty queue costs 16 workgroups that read one count
            const int rest_grid = (int)std::min<int64_t>(512, std::max<int64_t>(16, queued));
            DM_HIP(c, timed(KC_REST3 + (b - 3), s, [&] {
                     return launch_bin_rest(lb, pj, items, n, c->dq_list[i].p, c->dq_cnt[i].p, par, c->d_dq + i,
                                            rest_grid, gl, gc, done, s);
                   }),
                   "group kernel (dense split)");
            c->dq_par[i] ^= 1;
          }
          if (wb) DM_HIP(c, check_dense(c, i, b, j, s), "dense split check");
          continue;
        }
      }
      if (done) {  // (a tick in the one-kernel form carries no event: consumers join instead)
        c->tick_flagged = false;
        c->tick_part_mask = 0;
      }
      DM_HIP(c, timed(KC_BIN0 + b, s, [&] { return launch_bin(lb, pj, items, n, gl, gc, s); }), "group kernel");
      if (b >= 3 && b < 3 + dm_ctx::kSplitBins && wb) DM_HIP(c, check_dense(c, i, b, j, s), "dense split check");
    }
  }
  if (!c->h_tiles.empty())
    DM_HIP(c, timed(KC_SMALL, s_small, [&] { return launch_tile_small(p, c->tiles.p, c->tile_list.p, (int)c->h_tiles.size(), s_small); }),
           "small kernel");
  if (fork) {
    c->aux_pending = true;
    // k_general consumes every class's worklist appends on the context stream
    const bool defer = (flags & DM_ASYNC) && (flags & DM_DEFER_JOIN) && !general;
    if (!defer) DM_HIP(c, c->join_aux(), "join");
  }
  if (general) {
    const int blocks = (int)std::min<int64_t>(c->n_nonsmall, 1024);
    DM_HIP(c, timed(KC_GENERAL, st, [&] { return launch_general(p, gl, gc, blocks, st); }), "general kernel");
    c->main_dirty = true;
  }
  if (pingpong) std::swap(c->has, c->out_gets);  // the written column becomes the store's (stream order)
  c->last_writeback = wb;
  c->have_result = true;
  if (wb) c->hints_set = true;
  if (wb) c->expl_rows = false;
  c->chain_live_ok = wb && chain_live;
  if (!(flags & DM_ASYNC)) {
    rc = c->synced("tick");
    c->collect_profile();
    return rc;
  }
  return DM_OK;
}

// A round of requests, each decided by Resource.Decide in the caller's order and
// seeing the Assigns of the requests before it on the same resource
// (dm_round.hip).  Requests are ordered by resource on the host (stable: a
// resource's requests keep the caller's order); one workgroup per resource with
// requests, over a scratch copy of its rows.
int dm_decide(dm_ctx* c, int64_t now_ns, int64_t n, const int64_t* rows, const double* has, const double* wants,
              const int64_t* subclients, double* gets, int64_t* expiry_ns) {
  DM_ENTER(c);
  int rc = ready(c);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!rows || !has || !wants || !subclients || !gets || !expiry_ns)))
    return c->fail(DM_E_INVAL, "bad requests");
  if (n == 0) return DM_OK;
  c->expl_rows = true;  // decided rows take explicit expiries
  c->rows_changed();
  std::vector<int64_t> seg_of((size_t)n);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t r = rows[k];
    if (r < 0 || r >= c->N) return c->fail(DM_E_RANGE, "request row out of range");
    if (subclients[k] < 0 || subclients[k] > kSubMax) return c->fail(DM_E_INVAL, "subclients must be in [0, 2^31-2]");
    seg_of[(size_t)k] = std::upper_bound(c->h_seg_off.begin(), c->h_seg_off.end(), r) - c->h_seg_off.begin() - 1;
  }
  std::vector<int64_t> order((size_t)n);
  for (int64_t i = 0; i < n; ++i) order[(size_t)i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return seg_of[(size_t)a] < seg_of[(size_t)b]; });
  std::vector<int64_t> srows((size_t)n), ssub((size_t)n);
  std::vector<double> shas((size_t)n), swants((size_t)n);
  std::vector<ReqItem> items;
  int64_t scratch = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = order[(size_t)i], seg = seg_of[(size_t)k];
    srows[(size_t)i] = rows[k];
    shas[(size_t)i] = has[k];
    swants[(size_t)i] = wants[k];
    ssub[(size_t)i] = subclients[k];
    if (items.empty() || items.back().seg != (int32_t)seg) {
      items.push_back(ReqItem{(int32_t)seg, 0, i, i, scratch});
      scratch += c->h_seg_off[seg + 1] - c->h_seg_off[seg];
    }
    items.back().qhi = i + 1;
  }
  // Resources with many requests try the fast path (dm_decide_fast.hip): per request
  // the previous request of the round on the same row (its Assign is what the row
  // holds then), per resource its scan / sort areas.  The device decides whether the
  // round qualifies (FastRes::ok); k_decide takes every item it does not.
  std::vector<FastItem> fitems;
  std::vector<int64_t> prev;
  int64_t m_off = 0, e_off = 0, b_off = 0, c_off = 0;
  for (size_t ii = 0; c->decide_fast && ii < items.size(); ++ii) {
    ReqItem& itm = items[ii];
    const int64_t K = itm.qhi - itm.qlo;
    if (K < kFdMin) continue;
    if (prev.empty()) prev.assign((size_t)n, -1);
    FastItem f{};
    f.item = (int32_t)ii;
    f.k0 = itm.qlo;
    f.K = K;
    f.n = c->h_seg_off[itm.seg + 1] - c->h_seg_off[itm.seg];
    f.nblk = (int32_t)((K + kFdBlock - 1) / kFdBlock);
    f.m0 = m_off;
    f.e0 = e_off;
    f.b0 = b_off;
    f.c0 = c_off;
    f.nch = (int32_t)std::max<int64_t>(1, (f.n + kFdRows - 1) / kFdRows);
    m_off += f.n + 1;
    e_off += 2 * K;
    b_off += f.nblk;
    c_off += f.nch;
    itm.fast = (int32_t)fitems.size() + 1;
    fitems.push_back(f);
    std::unordered_map<int64_t, int64_t> last;
    last.reserve((size_t)(2 * K));
    for (int64_t k = itm.qlo; k < itm.qhi; ++k) {
      auto f2 = last.find(srows[(size_t)k]);
      if (f2 != last.end()) {
        prev[(size_t)k] = f2->second;
        fitems.back().repeats = 1;
      }
      last[srows[(size_t)k]] = k;
    }
  }
  hipStream_t st = c->stream;
  DM_HIP(c, upload(c->rq_rows, srows.data(), (size_t)n, st), "stage requests");
  DM_HIP(c, upload(c->rq_has, shas.data(), (size_t)n, st), "stage requests");
  DM_HIP(c, upload(c->rq_wants, swants.data(), (size_t)n, st), "stage requests");
  DM_HIP(c, upload(c->rq_sub, ssub.data(), (size_t)n, st), "stage requests");
  DM_HIP(c, upload(c->rq_items, items.data(), items.size(), st), "stage requests");
  DM_HIP(c, c->rq_gets.ensure((size_t)n), "request results");
  DM_HIP(c, c->rq_exp.ensure((size_t)n), "request results");
  DM_HIP(c, c->rq_sc_has.ensure((size_t)std::max<int64_t>(scratch, 1)), "request scratch");
  DM_HIP(c, c->rq_sc_wants.ensure((size_t)std::max<int64_t>(scratch, 1)), "request scratch");
  DM_HIP(c, c->rq_sc_sub.ensure((size_t)std::max<int64_t>(scratch, 1)), "request scratch");
  DevParams p{};
  p.seg_off = c->seg_off.p;
  p.wants = c->wants.p;
  p.has = c->has.p;
  p.sub = c->sub.p;
  p.expiry = c->expiry.p;
  p.cfg = c->cfg.p;
  p.agg = c->agg.p;
  p.expl = c->expl.p;
  p.now = now_ns;
  p.recompute = 0;
  const int nfast = (int)fitems.size();
  FastArgs fa{};
  const int64_t *d_eb = nullptr, *d_ee = nullptr;
  int neb = 0;
  size_t need = 0, need2 = 0;
  if (nfast > 0) {
    DM_HIP(c, upload(c->fd_items, fitems.data(), fitems.size(), st), "fast path");
    DM_HIP(c, upload(c->fd_prev, prev.data(), prev.size(), st), "fast path");
    DM_HIP(c, c->fd_res.ensure((size_t)nfast), "fast path");
    DM_HIP(c, c->fd_pw.ensure((size_t)n), "fast path");
    DM_HIP(c, c->fd_v.ensure((size_t)n), "fast path");
    DM_HIP(c, c->fd_sc.ensure((size_t)n), "fast path");
    DM_HIP(c, c->fd_keys.ensure((size_t)m_off), "fast path");
    DM_HIP(c, c->fd_keys_s.ensure((size_t)m_off), "fast path");
    DM_HIP(c, c->fd_ps.ensure((size_t)m_off), "fast path");
    DM_HIP(c, c->fd_ev_in.ensure((size_t)e_off), "fast path");
    DM_HIP(c, c->fd_evs_in.ensure((size_t)e_off), "fast path");
    DM_HIP(c, c->fd_ev.ensure((size_t)e_off), "fast path");
    DM_HIP(c, c->fd_evs.ensure((size_t)e_off), "fast path");
    DM_HIP(c, c->fd_ecnt.ensure((size_t)(b_off * (2 * kFdBlock + 1))), "fast path");
    DM_HIP(c, c->fd_esum.ensure((size_t)(b_off * (2 * kFdBlock + 1))), "fast path");
    DM_HIP(c, c->fd_bdc.ensure((size_t)b_off), "fast path");
    DM_HIP(c, c->fd_bds.ensure((size_t)b_off), "fast path");
    DM_HIP(c, c->fd_pc.ensure((size_t)c_off), "fast path");
    DM_HIP(c, c->fd_pt.ensure((size_t)c_off), "fast path");
    DM_HIP(c, c->fd_ld.ensure((size_t)n), "fast path");
    int64_t most = 1;
    for (const FastItem& f : fitems) most = std::max(most, std::max(f.K, f.n + 1));
    DM_HIP(c, c->fd_part.ensure((size_t)((most + kFdChunk - 1) / kFdChunk)), "fast path");
    // segment bounds of the event blocks' sort
    std::vector<int64_t> eb, ee;
    for (const FastItem& f : fitems)
      for (int64_t b = 0; b < f.nblk; ++b) {
        eb.push_back(f.e0 + 2 * b * kFdBlock);
        ee.push_back(f.e0 + 2 * std::min<int64_t>(f.K, (b + 1) * kFdBlock));
      }
    neb = (int)eb.size();
    std::vector<int64_t> bounds(eb);
    bounds.insert(bounds.end(), ee.begin(), ee.end());
    DM_HIP(c, upload(c->fd_bounds, bounds.data(), bounds.size(), st), "fast path");
    d_eb = c->fd_bounds.p;
    d_ee = d_eb + eb.size();
    fa = FastArgs{c->fd_items.p, c->fd_res.p,    c->fd_prev.p, c->fd_pw.p,    c->fd_v.p,      c->fd_sc.p,
                  c->fd_keys.p,  c->fd_keys_s.p, c->fd_ps.p,   c->fd_ev_in.p, c->fd_evs_in.p, c->fd_ev.p,
                  c->fd_evs.p,   c->fd_ecnt.p,   c->fd_esum.p, c->fd_bdc.p,   c->fd_bds.p,    c->fd_pc.p,
                  c->fd_pt.p,    c->fd_ld.p};
    for (const FastItem& f : fitems) {
      size_t b1 = 0;
      DM_HIP(c, fd_sort_keys(nullptr, &b1, c->fd_keys.p + f.m0, c->fd_keys_s.p + f.m0, f.n, st), "fast path");
      need = std::max(need, b1);
    }
    DM_HIP(c, fd_sort_pairs(nullptr, &need2, c->fd_ev_in.p, c->fd_ev.p, c->fd_evs_in.p, c->fd_evs.p, e_off, neb, d_eb,
                            d_ee, st),
           "fast path");
    DM_HIP(c, c->fd_tmp.ensure(std::max<size_t>(std::max(need, need2), 1)), "fast path");
  }
  const ReqArgs q{c->rq_rows.p, c->rq_has.p,     c->rq_wants.p,    c->rq_sub.p,   c->rq_gets.p,
                  c->rq_exp.p,  c->rq_sc_has.p,  c->rq_sc_wants.p, c->rq_sc_sub.p, nfast ? c->fd_res.p : nullptr};
  // the device work of the round (one profiling class: dm_kernel_times "decide")
  auto launches = [&]() -> hipError_t {
    hipError_t e = hipSuccess;
    if (nfast > 0) {
      for (int s2 = 0; s2 < nfast; ++s2) {
        const FastItem& f = fitems[(size_t)s2];
        if ((e = fd_rows(p, items[(size_t)f.item], f, s2, q, fa, st)) != hipSuccess) return e;
        if ((e = fd_item(p, items[(size_t)f.item], f, s2, q, fa, c->fd_part.p, st)) != hipSuccess) return e;
        size_t t1 = c->fd_tmp.n;
        if ((e = fd_sort_keys(c->fd_tmp.p, &t1, c->fd_keys.p + f.m0, c->fd_keys_s.p + f.m0, f.n, st)) != hipSuccess)
          return e;
      }
      size_t t2 = c->fd_tmp.n;
      if ((e = fd_sort_pairs(c->fd_tmp.p, &t2, c->fd_ev_in.p, c->fd_ev.p, c->fd_evs_in.p, c->fd_evs.p, e_off, neb,
                             d_eb, d_ee, st)) != hipSuccess)
        return e;
      for (int s2 = 0; s2 < nfast; ++s2)
        if ((e = fd_item_sorted(p, items[(size_t)fitems[(size_t)s2].item], fitems[(size_t)s2], s2, q, fa,
                                c->fd_part.p, st)) != hipSuccess)
          return e;
    }
    return launch_decide(p, c->rq_items.p, (int)items.size(), q, st);
  };
  DM_HIP(c, c->timed(KC_DECIDE, st, launches), "decide requests");
  DM_HIP(c, download(shas.data(), (const double*)c->rq_gets.p, 0, n, st), "read decisions");
  DM_HIP(c, download(ssub.data(), (const int64_t*)c->rq_exp.p, 0, n, st), "read decisions");
  if (int rs = c->synced("decide requests")) return rs;
  for (int64_t i = 0; i < n; ++i) {
    gets[order[(size_t)i]] = shas[(size_t)i];
    expiry_ns[order[(size_t)i]] = ssub[(size_t)i];
  }
  return DM_OK;
}

static int check_range(dm_ctx* c, int64_t off, int64_t n, int64_t total) {
  if (off < 0 || n < 0 || off + n > total) return c->fail(DM_E_RANGE, "range out of bounds");
  return DM_OK;
}

int dm_read_leases(dm_ctx* c, int64_t off, int64_t n, double* gets, int64_t* expiry_ns) {
  DM_ENTER(c);
  DM_STORE_READABLE(c);
  if (!c->have_result) return c->fail(DM_E_STATE, "no dm_apportion result");
  int rc = check_range(c, off, n, c->N);
  if (rc) return rc;
  DM_HIP(c, download(gets, c->last_writeback ? c->has.p : c->out_gets.p, off, n, c->stream), "read gets");
  if (expiry_ns && c->last_writeback) {  // the store's encoding, resolved on the device
    DM_HIP(c, c->st_exp.ensure((size_t)std::max<int64_t>(n, 1)), "stage expiry");
    DM_HIP(c, launch_resolve_rows(n, nullptr, off, c->sub.p, c->expiry.p, c->row_index(), c->agg.p, c->st_exp.p,
                                  nullptr, c->stream),
           "resolve expiry");
    DM_HIP(c, download(expiry_ns, (const int64_t*)c->st_exp.p, 0, n, c->stream), "read expiry");
  } else {
    DM_HIP(c, download(expiry_ns, (const int64_t*)c->out_expiry.p, off, n, c->stream), "read expiry");
  }
  return c->synced("read leases");
}

int dm_read_leases_rows(dm_ctx* c, int64_t n, const int64_t* rows, double* gets, int64_t* expiry_ns) {
  DM_ENTER(c);
  DM_STORE_READABLE(c);
  if (!c->have_result) return c->fail(DM_E_STATE, "no dm_apportion result");
  if (n < 0 || (n > 0 && !rows)) return c->fail(DM_E_INVAL, "bad rows");
  if (n == 0) return DM_OK;
  for (int64_t i = 0; i < n; ++i)
    if (rows[i] < 0 || rows[i] >= c->N) return c->fail(DM_E_RANGE, "row out of range");
  const double* g = c->last_writeback ? c->has.p : c->out_gets.p;
  const int64_t* e = c->last_writeback ? nullptr : c->out_expiry.p;  // the store's encoding: resolved below
  DM_HIP(c, c->st_rows.ensure((size_t)n), "stage rows");
  DM_HIP(c, c->st_has.ensure((size_t)n), "stage gets");
  DM_HIP(c, c->st_exp.ensure((size_t)n), "stage expiry");
  DM_HIP(c, hipMemcpyAsync(c->st_rows.p, rows, (size_t)n * 8, hipMemcpyHostToDevice, c->stream), "stage rows");
  DM_HIP(c, launch_gather_leases(n, c->st_rows.p, g, e, c->st_has.p, c->st_exp.p, c->stream), "gather leases");
  if (!e)
    DM_HIP(c, launch_resolve_rows(n, c->st_rows.p, 0, c->sub.p, c->expiry.p, c->row_index(), c->agg.p, c->st_exp.p,
                                  nullptr, c->stream),
           "resolve expiry");
  DM_HIP(c, download(gets, (const double*)c->st_has.p, 0, n, c->stream), "read gets");
  DM_HIP(c, download(expiry_ns, (const int64_t*)c->st_exp.p, 0, n, c->stream), "read expiry");
  return c->synced("read leases");
}

int dm_read_leases_proto(dm_ctx* c, int64_t off, int64_t n, double* capacity, int64_t* expiry_time_s,
                         int64_t* refresh_interval_s) {
  std::vector<int64_t> e(n > 0 ? n : 0);
  int rc = dm_read_leases(c, off, n, capacity, e.data());
  if (rc) return rc;
  if (expiry_time_s)
    for (int64_t i = 0; i < n; ++i) {
      // time.Time.Unix(): floor division by 1e9 (server.go:789)
      int64_t v = e[i];
      if (v == DM_RELEASED) {
        expiry_time_s[i] = DM_RELEASED;
        continue;
      }
      int64_t q = v / kNs;
      if (v % kNs != 0 && v < 0) --q;
      expiry_time_s[i] = q;
    }
  if (refresh_interval_s && n > 0) {
    // the device config: a hierarchy exchange rewrites a leaf's algorithm (dm_hier_root_tick)
    const auto& so = c->h_seg_off;
    const int64_t r0 = std::upper_bound(so.begin(), so.end(), off) - so.begin() - 1;
    const int64_t r1 = std::upper_bound(so.begin(), so.end(), off + n - 1) - so.begin() - 1;
    std::vector<ResCold> cf((size_t)(r1 - r0 + 1));
    DM_HIP(c, download(cf.data(), (const ResCold*)c->cold.p, r0, r1 - r0 + 1, c->stream), "read config");
    DM_HIP(c, hipStreamSynchronize(c->stream), "read config");
    int64_t r = r0;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t row = off + i;
      while (r + 1 < (int64_t)so.size() && so[r + 1] <= row) ++r;
      refresh_interval_s[i] = e[i] == DM_RELEASED ? 0 : cf[(size_t)(r - r0)].refresh_s;
    }
  }
  return DM_OK;
}

int dm_read_resources(dm_ctx* c, int64_t r0, int64_t n, int64_t* count, double* sum_has, double* sum_wants,
                      double* safe) {
  DM_ENTER(c);
  DM_STORE_READABLE(c);
  int rc = check_range(c, r0, n, c->R);
  if (rc) return rc;
  if (safe && !c->have_result) return c->fail(DM_E_STATE, "safe capacity needs a dm_apportion result");
  const bool wb = !c->have_result || c->last_writeback;
  std::vector<ResAgg> v(n > 0 ? n : 0);
  std::vector<ResCfg> cf(safe && n > 0 ? n : 0);
  std::vector<ResCold> cc(safe && n > 0 ? n : 0);
  DM_HIP(c, download(v.data(), (const ResAgg*)(wb ? c->agg.p : c->res.p), r0, n, c->stream), "read resources");
  // the device config: a hierarchy exchange rewrites a leaf's templates (dm_hier_root_tick)
  if (safe) DM_HIP(c, download(cf.data(), (const ResCfg*)c->cfg.p, r0, n, c->stream), "read config");
  if (safe) DM_HIP(c, download(cc.data(), (const ResCold*)c->cold.p, r0, n, c->stream), "read config");
  if (int rs = c->synced("read resources")) return rs;
  for (int64_t i = 0; i < n; ++i) {
    if (count) count[i] = v[i].count;
    if (sum_has) sum_has[i] = v[i].sum_has;
    if (sum_wants) sum_wants[i] = v[i].sum_wants;
    // SetSafeCapacity (resource.go:81-96) after the tick's Clean: configured, or capacity / Count
    if (safe) safe[i] = std::isnan(cc[i].safe_capacity) ? cf[i].capacity / (double)v[i].count : cc[i].safe_capacity;
  }
  return DM_OK;
}

int dm_read_config(dm_ctx* c, int64_t r0, int64_t n, int32_t* kind, double* capacity, int64_t* lease_length_s,
                   int64_t* refresh_interval_s, int64_t* learning_end_ns, int64_t* parent_expiry_ns,
                   double* safe_capacity) {
  DM_ENTER(c);
  if (!c->cfg_loaded) return c->fail(DM_E_STATE, "no configuration loaded");
  int rc = check_range(c, r0, n, c->R);
  if (rc) return rc;
  std::vector<ResCfg> v(n > 0 ? (size_t)n : 0);
  std::vector<ResCold> vc(n > 0 ? (size_t)n : 0);
  DM_HIP(c, download(v.data(), (const ResCfg*)c->cfg.p, r0, n, c->stream), "read config");
  DM_HIP(c, download(vc.data(), (const ResCold*)c->cold.p, r0, n, c->stream), "read config");
  DM_HIP(c, hipStreamSynchronize(c->stream), "read config");
  for (int64_t i = 0; i < n; ++i) {
    if (kind) kind[i] = v[i].kind;
    if (capacity) capacity[i] = v[i].capacity;
    if (lease_length_s) lease_length_s[i] = v[i].lease_len_s;
    if (refresh_interval_s) refresh_interval_s[i] = vc[i].refresh_s;
    if (learning_end_ns) learning_end_ns[i] = v[i].learning_end_ns;
    if (parent_expiry_ns) parent_expiry_ns[i] = v[i].parent_expiry_ns;
    if (safe_capacity) safe_capacity[i] = vc[i].safe_capacity;
  }
  return DM_OK;
}

int dm_read_store(dm_ctx* c, int64_t off, int64_t n, double* has, double* wants, int64_t* sub, int64_t* exp) {
  DM_ENTER(c);
  DM_STORE_READABLE(c);
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  int rc = check_range(c, off, n, c->N);
  if (rc) return rc;
  DM_HIP(c, download(has, (const double*)c->has.p, off, n, c->stream), "read has");
  DM_HIP(c, download(wants, (const double*)c->wants.p, off, n, c->stream), "read wants");
  if ((sub || exp) && n > 0) {  // subclients and expiry from the column encoding (dm_device.h)
    DM_HIP(c, c->st_exp.ensure((size_t)n), "stage expiry");
    DM_HIP(c, c->st_sub.ensure((size_t)n), "stage subclients");
    DM_HIP(c, launch_resolve_rows(n, nullptr, off, c->sub.p, c->expiry.p, c->row_index(), c->agg.p,
                                  exp ? c->st_exp.p : nullptr, sub ? c->st_sub.p : nullptr, c->stream),
           "resolve rows");
    DM_HIP(c, download(exp, (const int64_t*)c->st_exp.p, 0, n, c->stream), "read expiry");
    DM_HIP(c, download(sub, (const int64_t*)c->st_sub.p, 0, n, c->stream), "read subclients");
  }
  return c->synced("read store");
}

// Rows of one upsert/release call: in range and unique (a bitmap over the table,
// O(n + N/64)); the resource of each row is found on the device.
// The call's columns cross PCIe in chunks on an auxiliary stream while the
// context stream validates the chunks already there (k_check_rows: no O(n) host
// pass, so pinned buffers from dm_host_alloc go at full DMA rate).  The apply
// kernel then runs on the context stream; finish_update() maps the flags.
struct StageCol {
  void* dst;
  const void* src;
  size_t elem;
};
static constexpr int64_t kStageChunk = 1 << 22;  // rows per copy/validate step

static int staged_check(dm_ctx* c, int64_t n, const StageCol* cols, int ncols, bool check_wants, bool check_sub) {
  if (!c->row_bits.p || c->row_bits.n < (size_t)(c->N / 32 + 1)) {
    DM_HIP(c, c->row_bits.ensure((size_t)(c->N / 32 + 1)), "row bitmap");
    DM_HIP(c, hipMemsetAsync(c->row_bits.p, 0, c->row_bits.n * sizeof(uint32_t), c->stream), "row bitmap");
  }
  if (!c->upd_flags.p) {
    DM_HIP(c, c->upd_flags.ensure(1), "update flags");
    DM_HIP(c, hipHostMalloc((void**)&c->h_flags, sizeof(uint32_t), hipHostMallocDefault), "update flags");
  }
  DM_HIP(c, hipMemsetAsync(c->upd_flags.p, 0, sizeof(uint32_t), c->stream), "update flags");
  // Every call that reads the staging buffers (updates, dm_read_leases_rows) waits
  // for its kernels before it returns, so the copies need not wait for the context
  // stream: they overlap whatever is still running there (e.g. an asynchronous
  // tick), and each chunk's validation is ordered after that work and its copy.
  hipStream_t cp = c->cpy;
  int k = 0;
  for (int64_t off = 0; off < n; off += kStageChunk, ++k) {
    const int64_t m = std::min(kStageChunk, n - off);
    for (int j = 0; j < ncols; ++j)
      DM_HIP(c,
             hipMemcpyAsync((char*)cols[j].dst + off * cols[j].elem, (const char*)cols[j].src + off * cols[j].elem,
                            (size_t)m * cols[j].elem, hipMemcpyHostToDevice, cp),
             "stage update");
    hipEvent_t ev = c->ev_stage[k & 1];
    DM_HIP(c, hipEventRecord(ev, cp), "stage update");
    DM_HIP(c, hipStreamWaitEvent(c->stream, ev, 0), "stage update");
    DM_HIP(c, launch_check_rows(m, c->st_rows.p + off, c->N, c->row_bits.p, check_wants ? c->st_wants.p + off : nullptr,
                                check_sub ? c->st_sub.p + off : nullptr, nullptr, c->upd_flags.p, c->stream),
           "check rows");
  }
  return DM_OK;
}

// After the apply kernel: clear the bitmap, fetch the flags, wait (the call is
// synchronous on return, so the caller may free its buffers), map errors.
static int finish_update(dm_ctx* c, int64_t n, uint32_t* flags_out) {
  DM_HIP(c, launch_clear_rows(n, c->st_rows.p, c->N, c->row_bits.p, c->stream), "clear rows");
  DM_HIP(c, hipMemcpyAsync(c->h_flags, c->upd_flags.p, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream),
         "update flags");
  if (int rs = c->synced("update")) return rs;
  const uint32_t f = *c->h_flags;
  *flags_out = f;
  if (f & kUpdRange) return c->fail(DM_E_RANGE, "row out of range");
  if (f & kUpdDup) return c->fail(DM_E_INVAL, "rows must be unique within one call");
  if (f & kUpdSub) return c->fail(DM_E_INVAL, "subclients must be in [0, 2^31-2]");
  return DM_OK;
}

// A store update can make a store "maybe general" (a NaN wants, subclients other than
// one) after its plan chose stream parts, which plan_parts leaves out for a store
// that is general when planned.  The parts stay (ADVICE r5 asked which): a tick that
// may run k_general joins every class stream before it (dm_apportion: no deferred
// join), so k_general sees both parts' worklist appends, and the parts' own kernels
// leave a heterogeneous resource untouched for it
// (tests/test_parts_gpu.py::test_parts_store_turning_general_keeps_its_parts).
static int mark_maybe_general(dm_ctx* c) {
  c->maybe_general = true;
  return DM_OK;
}

int dm_store_upsert(dm_ctx* c, int64_t n, const int64_t* rows, const double* has, const double* wants,
                    const int64_t* sub, const int64_t* exp) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (n < 0 || (n > 0 && (!rows || !has || !wants || !sub || !exp))) return c->fail(DM_E_INVAL, "bad upsert");
  if (n == 0) return DM_OK;
  c->expl_rows = true;
  c->rows_changed();
  DM_HIP(c, c->st_rows.ensure((size_t)n), "stage rows");
  DM_HIP(c, c->st_has.ensure((size_t)n), "stage has");
  DM_HIP(c, c->st_wants.ensure((size_t)n), "stage wants");
  DM_HIP(c, c->st_sub.ensure((size_t)n), "stage sub");
  DM_HIP(c, c->st_exp.ensure((size_t)n), "stage expiry");
  const StageCol cols[] = {{c->st_rows.p, rows, 8}, {c->st_wants.p, wants, 8}, {c->st_sub.p, sub, 8},
                           {c->st_has.p, has, 8}, {c->st_exp.p, exp, 8}};
  int rc = staged_check(c, n, cols, 5, true, true);
  if (rc) return rc;
  DM_HIP(c, launch_upsert(n, c->st_rows.p, c->st_has.p, c->st_wants.p, c->st_sub.p, nullptr, c->st_exp.p, c->cfg.p, 0,
                          c->row_index(), c->has.p, c->wants.p, c->sub.p, c->expiry.p, c->agg.p, c->expl.p,
                          c->upd_flags.p, c->dense_upd(), c->stream),
         "upsert");
  uint32_t f = 0;
  rc = finish_update(c, n, &f);
  if (rc) return rc;
  // an upsert can make a resource's subclients heterogeneous: stay conservative
  if ((f & (kUpdNaN | kUpdNotOne)) || !c->all_sub_one)
    if (int rg = mark_maybe_general(c)) return rg;
  if (f & kUpdNotOne) c->all_sub_one = false;
  c->have_result = false;
  return DM_OK;
}

int dm_store_update_wants(dm_ctx* c, int64_t n, const int64_t* rows, const double* wants) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (n < 0 || (n > 0 && (!rows || !wants))) return c->fail(DM_E_INVAL, "bad update");
  if (n == 0) return DM_OK;
  c->rows_changed();  // a NaN wants ends a resource's dense state
  DM_HIP(c, c->st_rows.ensure((size_t)n), "stage rows");
  DM_HIP(c, c->st_wants.ensure((size_t)n), "stage wants");
  const StageCol cols[] = {{c->st_rows.p, rows, 8}, {c->st_wants.p, wants, 8}};
  int rc = staged_check(c, n, cols, 2, true, false);
  if (rc) return rc;
  DM_HIP(c, launch_update_wants(n, c->st_rows.p, c->st_wants.p, c->row_index(), c->sub.p, c->wants.p, c->agg.p,
                                c->upd_flags.p, c->stream),
         "update wants");
  uint32_t f = 0;
  rc = finish_update(c, n, &f);
  if (rc) return rc;
  if (f & kUpdNaN)
    if (int rg = mark_maybe_general(c)) return rg;
  c->have_result = false;
  return DM_OK;
}

// The same narrow Assign with the rows as a bit mask (one bit per row of
// [first_row, first_row + 64 nwords)) and the values packed in row order: at
// more than ~3% of the rows updated the mask is smaller than 8-B row indices.
int dm_store_update_wants_mask(dm_ctx* c, int64_t first_row, int64_t nwords, const uint64_t* mask, int64_t n,
                               const double* wants) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (first_row < 0 || (first_row & 63) || nwords < 0 || n < 0 || (nwords > 0 && !mask) || (n > 0 && !wants))
    return c->fail(DM_E_INVAL, "bad masked update (first_row must be a multiple of 64)");
  if (nwords == 0) return n == 0 ? DM_OK : c->fail(DM_E_INVAL, "packed values without a mask");
  if (first_row + 64 * (nwords - 1) >= c->N) return c->fail(DM_E_RANGE, "mask words past the store's end");
  c->rows_changed();  // a NaN wants ends a resource's dense state
  const int64_t nb = (nwords + 255) / 256;
  DM_HIP(c, c->st_mask.ensure((size_t)nwords), "stage mask");
  DM_HIP(c, c->st_wants.ensure((size_t)std::max<int64_t>(n, 1)), "stage wants");
  DM_HIP(c, c->st_blk.ensure((size_t)nb), "stage block sums");
  DM_HIP(c, c->st_wpre.ensure((size_t)nwords), "stage word offsets");
  if (!c->upd_flags.p) {
    DM_HIP(c, c->upd_flags.ensure(1), "update flags");
    DM_HIP(c, hipHostMalloc((void**)&c->h_flags, sizeof(uint32_t), hipHostMallocDefault), "update flags");
  }
  DM_HIP(c, hipMemsetAsync(c->upd_flags.p, 0, sizeof(uint32_t), c->stream), "update flags");
  // the copies overlap whatever still runs on the context's streams (staged_check)
  DM_HIP(c, hipMemcpyAsync(c->st_mask.p, mask, (size_t)nwords * 8, hipMemcpyHostToDevice, c->cpy), "stage mask");
  if (n > 0)
    DM_HIP(c, hipMemcpyAsync(c->st_wants.p, wants, (size_t)n * 8, hipMemcpyHostToDevice, c->cpy), "stage wants");
  DM_HIP(c, hipEventRecord(c->ev_stage[0], c->cpy), "stage update");
  DM_HIP(c, hipStreamWaitEvent(c->stream, c->ev_stage[0], 0), "stage update");
  DM_HIP(c, launch_update_wants_mask(nwords, c->st_mask.p, first_row, c->N, n, c->st_wants.p, c->st_blk.p,
                                     c->st_wpre.p, c->row_index(), c->sub.p, c->wants.p, c->agg.p, c->upd_flags.p,
                                     c->stream, 2, 0, INT64_MAX),
         "masked update");
  DM_HIP(c, hipMemcpyAsync(c->h_flags, c->upd_flags.p, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream),
         "update flags");
  if (int rs = c->synced("update")) return rs;
  const uint32_t f = *c->h_flags;
  if (f & kUpdRange) return c->fail(DM_E_RANGE, "mask bit past the store's end");
  if (f & kUpdCount) return c->fail(DM_E_INVAL, "packed values must match the mask's set bits");
  if (f & kUpdNaN)
    if (int rg = mark_maybe_general(c)) return rg;
  c->have_result = false;
  return DM_OK;
}

int dm_store_release(dm_ctx* c, int64_t n, const int64_t* rows) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (n < 0 || (n > 0 && !rows)) return c->fail(DM_E_INVAL, "bad release");
  if (n == 0) return DM_OK;
  c->rows_changed();
  DM_HIP(c, c->st_rows.ensure((size_t)n), "stage rows");
  const StageCol cols[] = {{c->st_rows.p, rows, 8}};
  int rc = staged_check(c, n, cols, 1, false, false);
  if (rc) return rc;
  DM_HIP(c, launch_release(n, c->st_rows.p, c->row_index(), c->has.p, c->wants.p, c->sub.p, c->expiry.p,
                           c->agg.p, c->expl.p, c->upd_flags.p, c->dense_upd(), c->stream),
         "release");
  uint32_t f = 0;
  rc = finish_update(c, n, &f);
  if (rc) return rc;
  c->have_result = false;
  return DM_OK;
}

// One round of updates: every part's columns cross PCIe back to back on the copy
// stream; each part is validated and applied on the context stream as soon as its
// columns have landed (overlapping the later parts' copies), in the order refresh,
// departures, arrivals.  A part whose validation fails is not applied, nor is any
// later part (k_carry_reject); earlier parts stay applied.
static int batch_args(dm_ctx* c, const dm_store_batch* b) {
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (!b) return c->fail(DM_E_INVAL, "null batch");
  const int64_t nw = b->wants_nwords, nm = b->wants_n, nr = b->release_n, nu = b->upsert_n;
  if (nw < 0 || nm < 0 || nr < 0 || nu < 0) return c->fail(DM_E_INVAL, "negative batch sizes");
  if (nw == 0 && nm > 0) return c->fail(DM_E_INVAL, "packed values without a mask");
  if (nw > 0) {
    const int64_t fr = b->wants_first_row;
    if (fr < 0 || (fr & 63) || !b->wants_mask || (nm > 0 && !b->wants))
      return c->fail(DM_E_INVAL, "bad masked update (first_row must be a multiple of 64)");
    if (fr + 64 * (nw - 1) >= c->N) return c->fail(DM_E_RANGE, "mask words past the store's end");
  }
  if (nr > 0 && !b->release_rows) return c->fail(DM_E_INVAL, "bad release");
  // narrow arrivals: subclients as int32, has NULL (= 0), expiry NULL (= now + lease length)
  const bool sub32 = b->upsert_subclients32 != nullptr;
  if (nu > 0 && (!b->upsert_rows || !b->upsert_wants || (!b->upsert_subclients && !sub32)))
    return c->fail(DM_E_INVAL, "bad upsert");
  if (nu > 0 && !b->upsert_expiry_ns && !c->cfg_loaded)
    return c->fail(DM_E_STATE, "arrivals without expiries take the resource's lease length: load a configuration");
  if (nu > 0 && !b->upsert_expiry_ns && b->upsert_now_ns <= 0)  // an unset clock would insert lapsed leases
    return c->fail(DM_E_INVAL, "arrivals without expiries need upsert_now_ns (> 0): their expiry is now + lease length");
  return DM_OK;
}

// The batch's copies (copy stream), its three parts' kernels (context stream) and the
// flags' copy back into S.h_flags; nothing waits for them here.
static int apply_enqueue(dm_ctx* c, const dm_store_batch* b, dm_ctx::ApplySet& S) {
  const int64_t nw = b->wants_nwords, nm = b->wants_n, nr = b->release_n, nu = b->upsert_n;
  const bool sub32 = b->upsert_subclients32 != nullptr;
  if (nu > 0) c->expl_rows = true;  // arrivals take explicit expiries
  if (nu > 0 || nr > 0) c->chain_live_ok = false;  // subclients words written, rows released
  c->rows_changed();  // (wants refreshes too: a NaN wants ends a resource's dense state)
  S.nu = nu;
  hipStream_t st = c->stream, cp = c->cpy;
  if (!S.flags.p) {
    DM_HIP(c, S.flags.ensure(3), "batch flags");
    DM_HIP(c, hipHostMalloc((void**)&S.h_flags, 3 * sizeof(uint32_t), hipHostMallocDefault), "batch flags");
  }
  if (!c->row_bits.p || c->row_bits.n < (size_t)(c->N / 32 + 1)) {
    DM_HIP(c, c->row_bits.ensure((size_t)(c->N / 32 + 1)), "row bitmap");
    DM_HIP(c, hipMemsetAsync(c->row_bits.p, 0, c->row_bits.n * sizeof(uint32_t), st), "row bitmap");
  }
  DM_HIP(c, hipMemsetAsync(S.flags.p, 0, 3 * sizeof(uint32_t), st), "batch flags");
  uint32_t* F = S.flags.p;
  // the refresh's packed values cross in up to kWChunks chunks of >= 2^21 values, so
  // that the synchronous call's apply overlaps its own copies; an asynchronous batch's
  // apply overlaps the next batch's copies anyway, and one copy costs less than four
  // (C4 2.95 -> 2.91 ms per step, alternated: tools/archive/gpu_r6_c4chunk.sh)
  const bool sync_set = &S == &c->aset[0];
  const int nchunk = nw == 0 ? 0 : !sync_set ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>(dm_ctx::kWChunks, nm >> 21));
  // copies, back to back
  if (nw > 0) {
    DM_HIP(c, S.mask.ensure((size_t)nw), "stage mask");
    DM_HIP(c, S.mwants.ensure((size_t)std::max<int64_t>(nm, 1)), "stage wants");
    DM_HIP(c, S.blk.ensure((size_t)((nw + 255) / 256)), "stage block sums");
    DM_HIP(c, S.wpre.ensure((size_t)nw), "stage word offsets");
    DM_HIP(c, hipMemcpyAsync(S.mask.p, b->wants_mask, (size_t)nw * 8, hipMemcpyHostToDevice, cp), "stage mask");
    DM_HIP(c, hipEventRecord(S.ev_bat[0], cp), "stage");
    // the packed values in chunks, each applied as soon as it has landed (the apply
    // of one chunk overlaps the next one's copy): C4 3.2 -> ~3.0 ms per step
    for (int k = 0; k < nchunk; ++k) {
      const int64_t v0 = nm * k / nchunk, v1 = nm * (k + 1) / nchunk;
      if (v1 > v0)
        DM_HIP(c, hipMemcpyAsync(S.mwants.p + v0, b->wants + v0, (size_t)(v1 - v0) * 8, hipMemcpyHostToDevice, cp),
               "stage wants");
      DM_HIP(c, hipEventRecord(S.ev_wchunk[k], cp), "stage");
    }
  }
  if (nr > 0) {
    DM_HIP(c, S.rel.ensure((size_t)nr), "stage release rows");
    DM_HIP(c, hipMemcpyAsync(S.rel.p, b->release_rows, (size_t)nr * 8, hipMemcpyHostToDevice, cp), "stage rows");
    DM_HIP(c, hipEventRecord(S.ev_bat[1], cp), "stage");
  }
  if (nu > 0) {
    DM_HIP(c, S.rows.ensure((size_t)nu), "stage rows");
    DM_HIP(c, S.has.ensure((size_t)nu), "stage has");
    DM_HIP(c, S.wants.ensure((size_t)nu), "stage wants");
    DM_HIP(c, S.sub.ensure((size_t)nu), "stage sub");
    DM_HIP(c, S.exp.ensure((size_t)nu), "stage expiry");
    const StageCol cols[] = {{S.rows.p, b->upsert_rows, 8},
                             {S.wants.p, b->upsert_wants, 8},
                             {S.sub.p, sub32 ? (const void*)b->upsert_subclients32 : b->upsert_subclients, sub32 ? 4u : 8u},
                             {S.has.p, b->upsert_has, 8},
                             {S.exp.p, b->upsert_expiry_ns, 8}};
    for (const auto& col : cols)
      if (col.src)
        DM_HIP(c, hipMemcpyAsync(col.dst, col.src, (size_t)nu * col.elem, hipMemcpyHostToDevice, cp), "stage upsert");
    DM_HIP(c, hipEventRecord(S.ev_bat[2], cp), "stage");
  }
  // part 1: wants refresh (validated by its count/scan passes over the mask, then
  // applied chunk by chunk as the values land)
  if (nw > 0) {
    DM_HIP(c, hipStreamWaitEvent(st, S.ev_bat[0], 0), "stage");
    DM_HIP(c, launch_update_wants_mask(nw, S.mask.p, b->wants_first_row, c->N, nm, S.mwants.p, S.blk.p, S.wpre.p,
                                       c->row_index(), c->sub.p, c->wants.p, c->agg.p, F + 0, st, 0, 0, 0),
           "masked update");
    for (int k = 0; k < nchunk; ++k) {
      const int64_t v0 = nm * k / nchunk, v1 = nm * (k + 1) / nchunk;
      DM_HIP(c, hipStreamWaitEvent(st, S.ev_wchunk[k], 0), "stage");
      if (v1 > v0)
        DM_HIP(c, launch_update_wants_mask(nw, S.mask.p, b->wants_first_row, c->N, nm, S.mwants.p, S.blk.p, S.wpre.p,
                                           c->row_index(), c->sub.p, c->wants.p, c->agg.p, F + 0, st, 1, v0, v1),
               "masked update");
    }
  }
  // part 2: departures
  if (nr > 0) {
    DM_HIP(c, hipStreamWaitEvent(st, S.ev_bat[1], 0), "stage");
    DM_HIP(c, launch_check_rows(nr, S.rel.p, c->N, c->row_bits.p, nullptr, nullptr, nullptr, F + 1, st), "check rows");
    DM_HIP(c, launch_carry_reject(F + 0, F + 1, st), "carry");
    DM_HIP(c, launch_release(nr, S.rel.p, c->row_index(), c->has.p, c->wants.p, c->sub.p, c->expiry.p, c->agg.p,
                             c->expl.p, F + 1, c->dense_upd(), st),
           "release");
    DM_HIP(c, launch_clear_rows(nr, S.rel.p, c->N, c->row_bits.p, st), "clear rows");
  } else {
    DM_HIP(c, launch_carry_reject(F + 0, F + 1, st), "carry");
  }
  // part 3: arrivals / full refreshes
  if (nu > 0) {
    DM_HIP(c, hipStreamWaitEvent(st, S.ev_bat[2], 0), "stage");
    const int64_t* s64 = sub32 ? nullptr : S.sub.p;
    const int32_t* s32 = sub32 ? (const int32_t*)S.sub.p : nullptr;
    DM_HIP(c, launch_check_rows(nu, S.rows.p, c->N, c->row_bits.p, S.wants.p, s64, s32, F + 2, st), "check rows");
    DM_HIP(c, launch_carry_reject(F + 1, F + 2, st), "carry");
    DM_HIP(c, launch_upsert(nu, S.rows.p, b->upsert_has ? S.has.p : nullptr, S.wants.p, s64, s32,
                            b->upsert_expiry_ns ? S.exp.p : nullptr, c->cfg.p, b->upsert_now_ns, c->row_index(),
                            c->has.p, c->wants.p, c->sub.p, c->expiry.p, c->agg.p, c->expl.p, F + 2, c->dense_upd(), st),
           "upsert");
    DM_HIP(c, launch_clear_rows(nu, S.rows.p, c->N, c->row_bits.p, st), "clear rows");
  }
  DM_HIP(c, hipMemcpyAsync(S.h_flags, F, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "batch flags");
  c->have_result = false;
  return DM_OK;
}

// A landed batch's flags: the first rejected part fails the call (its message names the
// part; `late` marks an asynchronous batch reported by a later call), NaN wants or
// other subclient counts make the store maybe-general.
static int apply_check(dm_ctx* c, const dm_ctx::ApplySet& S, bool late) {
  const uint32_t f0 = S.h_flags[0], f1 = S.h_flags[1], f2 = S.h_flags[2];
  auto reject = [&](uint32_t f, const char* part) -> int {
    const std::string p = std::string(late ? "an earlier asynchronous batch's " : "") + part;
    if (f & kUpdRange) return c->fail(DM_E_RANGE, p + ": row out of range");
    if (f & kUpdCount) return c->fail(DM_E_INVAL, p + ": packed values must match the mask's set bits");
    if (f & kUpdDup) return c->fail(DM_E_INVAL, p + ": rows must be unique within one part");
    return c->fail(DM_E_INVAL, p + ": subclients must be in [0, 2^31-2]");
  };
  if (f0 & kUpdReject) return reject(f0, "wants refresh");
  if (f0 & kUpdNaN)
    if (int rg = mark_maybe_general(c)) return rg;
  if (f1 & kUpdReject) return reject(f1, "release");
  if (f2 & kUpdReject) return reject(f2, "upsert");
  if (S.nu > 0) {
    if ((f2 & (kUpdNaN | kUpdNotOne)) || !c->all_sub_one)
      if (int rg = mark_maybe_general(c)) return rg;
    if (f2 & kUpdNotOne) c->all_sub_one = false;
  }
  return DM_OK;
}

int dm_store_apply(dm_ctx* c, const dm_store_batch* b) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (int rc = batch_args(c, b)) return rc;
  if (b->wants_nwords == 0 && b->release_n == 0 && b->upsert_n == 0) return DM_OK;
  dm_ctx::ApplySet& S = c->aset[0];
  if (int rc = apply_enqueue(c, b, S)) return rc;
  if (int rs = c->synced("batch")) return rs;
  return apply_check(c, S, false);
}

// Retire asynchronous set S: wait for its batch, then its flags.
static int async_retire(dm_ctx* c, dm_ctx::ApplySet& S) {
  if (!S.pending) return DM_OK;
  const hipError_t e = hipEventSynchronize(S.ev_done);
  S.pending = false;
  if (e != hipSuccess) return c->fail(DM_E_HIP, std::string("asynchronous batch: ") + hipGetErrorString(e));
  return apply_check(c, S, true);
}

int dm_store_apply_async(dm_ctx* c, const dm_store_batch* b) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (int rc = batch_args(c, b)) return rc;
  if (b->wants_nwords == 0 && b->release_n == 0 && b->upsert_n == 0) return DM_OK;
  dm_ctx::ApplySet& S = c->aset[1 + (int)(c->async_seq % dm_ctx::kAsyncSets)];
  // the set's previous batch (kAsyncSets batches back) first: its flags, and its
  // staging free for these copies (this wait is what keeps the host kAsyncSets
  // batches ahead of the device at most)
  if (int rc = async_retire(c, S)) return rc;
  S.may_general = b->wants_nwords > 0 || b->upsert_n > 0;
  if (int rc = apply_enqueue(c, b, S)) return rc;
  DM_HIP(c, hipEventRecord(S.ev_done, c->stream), "batch done");
  S.pending = true;
  c->async_seq += 1;
  return DM_OK;
}

int dm_store_apply_wait(dm_ctx* c) {
  DM_ENTER(c);
  int first = DM_OK;
  std::string msg;
  for (int64_t k = c->async_seq - dm_ctx::kAsyncSets; k < c->async_seq; ++k) {  // oldest first
    if (k < 0) continue;
    const int rc = async_retire(c, c->aset[1 + (int)(k % dm_ctx::kAsyncSets)]);
    if (rc && first == DM_OK) {
      first = rc;
      msg = c->err;
    }
  }
  if (first != DM_OK) c->err = msg;
  return first;
}

int dm_host_alloc(dm_ctx* c, size_t bytes, void** out) {
  DM_CHECK_CTX(c);
  if (!out) return c->fail(DM_E_INVAL, "null out");
  *out = nullptr;
  if (bytes == 0) return DM_OK;
  DM_HIP(c, hipHostMalloc(out, bytes, hipHostMallocDefault), "pinned host buffer");
  return DM_OK;
}

int dm_host_free(dm_ctx* c, void* p) {
  DM_CHECK_CTX(c);
  if (p) DM_HIP(c, hipHostFree(p), "pinned host buffer");
  return DM_OK;
}

int dm_aggregate_bands(const double* wants, const int64_t* num_clients, int64_t n, double* wants_total,
                       int64_t* subclients_total) {
  if (n < 0 || (n > 0 && (!wants || !num_clients)) || !wants_total || !subclients_total) return DM_E_INVAL;
  double wt = 0.0;
  int64_t stot = 0;
  for (int64_t i = 0; i < n; ++i) {
    wt += wants[i];
    if (num_clients[i] < 1) {
      g_last_error = "subclients should be > 0";
      return DM_E_ARGUMENT;
    }
    stot += num_clients[i];
  }
  *wants_total = wt;
  *subclients_total = stot;
  return DM_OK;
}

int dm_publish_totals(dm_ctx* c, void* dst) {
  DM_ENTER(c);
  DM_STORE_OK(c);
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  if (!dst) return c->fail(DM_E_INVAL, "null destination");
  if (!c->pub_sync.p) {
    DM_HIP(c, c->pub_sync.ensure(2), "publish state");
    DM_HIP(c, hipMemsetAsync(c->pub_sync.p, 0, 2 * sizeof(uint32_t), c->stream), "publish state");
  }
  DM_HIP(c, c->timed(KC_PUBLISH, c->stream, [&] { return launch_publish(c->R, c->agg.p, dst, c->pub_sync.p, c->stream); }),
         "publish");
  return DM_OK;
}

int dm_publish_ring(dm_ctx* c, int n, void* const* bufs) {
  DM_ENTER(c);
  if (n < 0 || (n > 0 && !bufs)) return c->fail(DM_E_INVAL, "bad publish ring");
  if (n > 0 && n < 3) return c->fail(DM_E_INVAL, "a publish ring needs at least 3 buffers");
  for (int i = 0; i < n; ++i)
    if (!bufs[i]) return c->fail(DM_E_INVAL, "null publish buffer");
  c->pub_ring.clear();
  for (int i = 0; i < n; ++i) c->pub_ring.push_back((double2*)bufs[i]);
  c->pub_k = 0;
  // every buffer's record 0 starts clear: a tick clears only its own flags words of
  // the next buffer (DevParams::pub_word)
  for (int i = 0; i < n; ++i) DM_HIP(c, hipMemsetAsync(bufs[i], 0, sizeof(double2), c->stream), "publish ring");
  if (n > 0) c->main_dirty = true;
  return DM_OK;
}

int dm_hier_layout(dm_ctx* root, int n_servers, const int64_t* shard_lo, int64_t stride) {
  DM_ENTER(root);
  if (n_servers <= 0 || n_servers > kHierMaxServers) return root->fail(DM_E_INVAL, "1..64 intermediate servers");
  if (!root->store_loaded) return root->fail(DM_E_STATE, "load the root store first");
  int64_t widest = root->R;
  if (shard_lo) {
    if (shard_lo[0] != 0 || shard_lo[n_servers] != root->R)
      return root->fail(DM_E_INVAL, "shard bounds must run from 0 to the root's resource count");
    widest = 0;
    for (int g = 0; g < n_servers; ++g) {
      if (shard_lo[g + 1] < shard_lo[g]) return root->fail(DM_E_INVAL, "shard bounds must be non-decreasing");
      widest = std::max(widest, shard_lo[g + 1] - shard_lo[g]);
    }
  }
  if (stride == 0) stride = 1 + widest;
  if (stride < 1 + widest) return root->fail(DM_E_INVAL, "record stride below 1 + the largest shard");
  root->hier_G = n_servers;
  root->hier_sharded = shard_lo != nullptr;
  root->hier_stride = stride;
  if (shard_lo) {
    root->h_hier_lo.assign(shard_lo, shard_lo + n_servers + 1);
    DM_HIP(root, upload(root->hier_lo, root->h_hier_lo.data(), root->h_hier_lo.size(), root->stream), "shard bounds");
  } else {
    root->h_hier_lo.clear();
  }
  return DM_OK;
}

int dm_hier_pipeline(dm_ctx* leaf, int on) {
  DM_ENTER(leaf);
  if (!leaf->cfg_loaded) return leaf->fail(DM_E_STATE, "load the leaf's configuration first");
  if (on < 0 || on > dm_ctx::kTplSlots - 1) return leaf->fail(DM_E_INVAL, "pipeline lag must be 0..3");
  if (!on && leaf->tpl_pipe && !leaf->tpl_pending.empty()) {  // take the newest staged templates now
    const int take = leaf->tpl_pending.back().slot;
    DM_HIP(leaf, leaf->xs_wait(leaf->tpl_ready[take], leaf->stream), "staged templates");
    std::swap(leaf->cfg, leaf->tpl_cfg[take]);
    std::swap(leaf->cold, leaf->tpl_cold[take]);
  }
  leaf->tpl_pending.clear();
  leaf->tpl_free_slots.clear();
  for (int i = 0; i < dm_ctx::kTplSlots; ++i) {
    leaf->tpl_free_slots.push_back(i);
    leaf->tpl_free_rec[i] = false;
  }
  if (on) DM_HIP(leaf, hipStreamSynchronize(leaf->stream), "template slots");  // no tick still reads a slot
  leaf->tpl_pipe = on != 0;
  leaf->tpl_lag = on > 1 ? on : 1;
  return DM_OK;
}

// One exchange round of the hierarchy (server.go:227-323 -> :822-901): decide the
// round on the root store from every server's published block (the request and
// its validation flags, dm_publish_totals) and write this server's templates into
// its leaf -- in place, or into a staged slot the leaf takes one tick later
// (dm_hier_pipeline).  Stream-ordered: the all-gather that produced `gathered`
// must precede it on the root's stream.
// The exchange's stream after leaf tick `seq`: its parts' events (dm_ctx::tick_ev).
static hipError_t wait_tick(dm_ctx* leaf, uint64_t seq, hipStream_t s) {
  const int k = (int)(seq % dm_ctx::kTickEv);
  for (int j = 0; j < std::max(leaf->tick_nev[k], 1); ++j) {
    hipError_t e = hipStreamWaitEvent(s, leaf->tick_ev[j][k], 0);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int dm_hier_root_tick(dm_ctx* root, const void* gathered, int n_servers, int64_t now_ns, dm_ctx* leaf, int server) {
  DM_ENTER(root);
  DM_STORE_OK(root);
  if (!root->store_loaded || !root->cfg_loaded) return root->fail(DM_E_STATE, "root store / config not loaded");
  if (!gathered || !leaf) return root->fail(DM_E_INVAL, "null gathered buffer or leaf context");
  if (n_servers <= 0 || n_servers > kHierMaxServers)
    return root->fail(DM_E_INVAL, "1..64 intermediate servers per root store");
  if (root->hier_G != 0 && root->hier_G != n_servers)
    return root->fail(DM_E_INVAL, "n_servers differs from the root's dm_hier_layout");
  const bool sharded = root->hier_G != 0 && root->hier_sharded;
  const int K = sharded ? 1 : n_servers;
  root->expl_rows = true;  // the root's rows take the exchange's explicit expiries
  root->rows_changed();
  // checked at load (seg_uniform), not per round
  if (root->R <= 0 || root->N != root->R * (int64_t)K || root->seg_uniform != K)
    return root->fail(DM_E_STATE, sharded ? "sharded root store must hold one row per resource"
                                          : "root store must hold R resources x n_servers rows (resource r: rows "
                                            "r*G..r*G+G-1)");
  if (server < 0 || server >= n_servers) return root->fail(DM_E_RANGE, "server index out of range");
  if (leaf->device != root->device) return root->fail(DM_E_INVAL, "root and leaf contexts must share a device");
  const int64_t leaf_lo = sharded ? root->h_hier_lo[server] : 0;
  const int64_t leaf_R = sharded ? root->h_hier_lo[server + 1] - leaf_lo : root->R;
  if (!leaf->cfg_loaded || leaf->R != leaf_R)
    return root->fail(DM_E_STATE, "the leaf must hold exactly this server's resources");
  const int64_t stride = root->hier_G != 0 ? root->hier_stride : 1 + root->R;
  const bool same = root->stream == leaf->stream;
  // A pipelined leaf whose last tick's events cover its streams stays unjoined (the
  // round writes a free template slot, and waits on those events); otherwise the leaf's
  // streams join first.
  const bool cover = !same && leaf->tpl_pipe && leaf->tick_covers();
  if (!cover) {
    DM_HIP(root, leaf->join_aux(), "join leaf streams");
    leaf->main_dirty = true;
  }
  DM_HIP(root, root->hier_status.ensure((size_t)kHierMaxServers), "hierarchy status");
  root->hier_servers = n_servers;
  if (!same && !root->hs_ordered) {  // the root round after the leaf's prior work (its publish)
    if (cover) DM_HIP(root, wait_tick(leaf, leaf->tick_seq, root->stream), "leaf->root order");
    else DM_HIP(root, leaf->xs_order(dm_ctx::XS_LEAF, leaf->stream, root->stream), "leaf->root order");
  }
  ResCfg* tcfg = leaf->cfg.p;
  ResCold* tcold = leaf->cold.p;
  const ResCfg* pcfg = leaf->cfg.p;
  const ResCold* pcold = leaf->cold.p;
  int slot = -1;
  if (leaf->tpl_pipe) {
    if (leaf->tpl_free_slots.empty())
      return root->fail(DM_E_STATE, "too many staged exchanges: tick the leaf between exchanges");
    slot = leaf->tpl_free_slots.front();
    DM_HIP(root, leaf->tpl_cfg[slot].ensure((size_t)leaf->R), "template slot");
    DM_HIP(root, leaf->tpl_cold[slot].ensure((size_t)leaf->R), "template slot");
    if (leaf->stream != root->stream) leaf->tick_signal_wanted = true;
    if (leaf->stream == root->stream) {
      // stream order: the ticks that read the slot's old templates precede this round
    } else if (leaf->tpl_free_rec[slot] && leaf->tpl_free_seq[slot] > 0) {  // the ticks that read the slot's old
      if (cover && root->hs_ordered && leaf->tpl_free_seq[slot] <= leaf->tick_seq) {  // templates are done
        // this round already waits for the leaf's last tick, whose events cover every
        // earlier tick on the same streams
      } else if (leaf->tick_seq - leaf->tpl_free_seq[slot] < (uint64_t)dm_ctx::kTickEv - 1) {
        DM_HIP(root, wait_tick(leaf, leaf->tpl_free_seq[slot], root->stream), "template slot");
      } else {  // that tick's events were recorded again since: everything the leaf holds
        DM_HIP(root, leaf->join_aux(), "join leaf streams");
        leaf->main_dirty = true;
        DM_HIP(root, leaf->xs_order(dm_ctx::XS_LEAF, leaf->stream, root->stream), "template slot");
      }
    }
    else if (leaf->tpl_free_rec[slot])
      DM_HIP(root, leaf->xs_wait(leaf->tpl_free[slot], root->stream), "template slot");
    tcfg = leaf->tpl_cfg[slot].p;
    tcold = leaf->tpl_cold[slot].p;
    if (!leaf->tpl_pending.empty()) {  // a rejected round keeps the newest staged templates
      pcfg = leaf->tpl_cfg[leaf->tpl_pending.back().slot].p;
      pcold = leaf->tpl_cold[leaf->tpl_pending.back().slot].p;
    }
  }
  DevParams p{};
  p.seg_off = root->seg_off.p;
  p.wants = root->wants.p;
  p.has = root->has.p;
  p.sub = root->sub.p;
  p.expiry = root->expiry.p;
  p.cfg = root->cfg.p;
  p.agg = root->agg.p;
  p.expl = root->expl.p;
  p.out_gets = root->has.p;
  p.out_expiry = root->expiry.p;
  p.out_wants = root->wants.p;
  p.out_sub = root->sub.p;
  p.res = root->agg.p;
  p.now = now_ns;
  p.recompute = 0;  // the root's running sums, updated as the reference's Clean + Assigns
  HierArgs ha{};
  ha.gathered = (const double2*)gathered;
  ha.stride = stride;
  ha.shard_lo = sharded ? root->hier_lo.p : nullptr;
  ha.status_out = root->hier_status.p;
  ha.leaf_cfg = tcfg;
  ha.leaf_cold = tcold;
  ha.leaf_prev_cfg = pcfg;
  ha.leaf_prev_cold = pcold;
  ha.root_cold = root->cold.p;
  ha.R = root->R;
  ha.leaf_lo = leaf_lo;
  // Sharded: only this server ever requests its resources (server.go:234-255), and its
  // leaf reads only their templates, so the round is decided over its own range; the
  // root copy's other rows are the other ranks' (each decides its own range).
  ha.r_lo = sharded ? leaf_lo : 0;
  ha.r_hi = sharded ? leaf_lo + leaf_R : root->R;
  ha.G = n_servers;
  ha.K = K;
  ha.server = server;
  DM_HIP(root, root->timed(KC_HIER_ROOT, root->stream, [&] { return launch_hier_tick(p, ha, root->stream); }),
         "hierarchy root tick");
  if (slot >= 0) {
    leaf->tpl_free_slots.erase(leaf->tpl_free_slots.begin());
    if (same)  // the leaf's ticks follow in stream order
      leaf->xs_signal_lazy(dm_ctx::XS_READY0 + slot, root->stream, &leaf->tpl_ready[slot]);
    else
      DM_HIP(root,
             leaf->xs_signal(dm_ctx::XS_READY0 + slot, root->stream, &leaf->tpl_ready[slot]),
             "staged templates");
    leaf->tpl_pending.push_back(dm_ctx::Staged{slot, leaf->ticks_issued});
  } else if (!same) {  // the leaf's next tick after its new templates
    DM_HIP(root, leaf->xs_order(dm_ctx::XS_ROOT, root->stream, leaf->stream), "root->leaf order");
  }
  root->maybe_general = true;  // rows carry heterogeneous subclient counts
  root->all_sub_one = false;
  root->last_writeback = true;
  root->have_result = true;
  return DM_OK;
}

// librccl, loaded on first use: the copy torch already mapped if there is one (one
// RCCL per process), else ROCm's
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};
static const RcclApi* rccl_api() {
  static RcclApi api;
  static bool tried = false;
  if (!tried) {
    tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if ((api.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
    for (int i = 0; !api.h && i < 3; ++i) api.h = dlopen(names[i], RTLD_NOW);
    if (api.h) {
      api.get_unique_id = (decltype(api.get_unique_id))dlsym(api.h, "ncclGetUniqueId");
      api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(api.h, "ncclCommInitRank");
      api.all_gather = (decltype(api.all_gather))dlsym(api.h, "ncclAllGather");
      api.comm_destroy = (decltype(api.comm_destroy))dlsym(api.h, "ncclCommDestroy");
      api.error_string = (decltype(api.error_string))dlsym(api.h, "ncclGetErrorString");
      api.comm_count = (decltype(api.comm_count))dlsym(api.h, "ncclCommCount");
      api.comm_user_rank = (decltype(api.comm_user_rank))dlsym(api.h, "ncclCommUserRank");
      if (!api.get_unique_id || !api.comm_init_rank || !api.all_gather || !api.comm_destroy || !api.error_string ||
          !api.comm_count || !api.comm_user_rank)
        api.h = nullptr;
    }
  }
  return api.h ? &api : nullptr;
}
static void rccl_destroy(const RcclApi* r, ncclComm_t comm) {
  if (r && comm) (void)r->comm_destroy(comm);
}

int dm_rccl_unique_id(void* id_out) {
  if (!id_out) return DM_E_INVAL;
  const RcclApi* r = rccl_api();
  if (!r) {
    g_last_error = "librccl not found";
    return DM_E_STATE;
  }
  ncclUniqueId id;
  const ncclResult_t e = r->get_unique_id(&id);
  if (e != ncclSuccess) {
    g_last_error = std::string("ncclGetUniqueId: ") + r->error_string(e);
    return DM_E_HIP;
  }
  memcpy(id_out, &id, sizeof id);
  return DM_OK;
}

int dm_hier_comm_init(dm_ctx* root, const void* id, int nranks, int rank) {
  DM_ENTER(root);
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return root->fail(DM_E_INVAL, "bad communicator arguments");
  if (root->nccl_comm) return root->fail(DM_E_STATE, "the exchange already has a communicator");
  const RcclApi* r = rccl_api();
  if (!r) return root->fail(DM_E_STATE, "librccl not found");
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  const ncclResult_t e = r->comm_init_rank(&root->nccl_comm, nranks, uid, rank);
  if (e != ncclSuccess) {
    root->nccl_comm = nullptr;
    return root->fail(DM_E_HIP, std::string("ncclCommInitRank: ") + r->error_string(e));
  }
  return DM_OK;
}

int dm_hier_comm_info(dm_ctx* root, int* nranks, int* rank) {
  DM_CHECK_CTX(root);
  if (!nranks || !rank) return root->fail(DM_E_INVAL, "null output");
  if (!root->nccl_comm) return root->fail(DM_E_STATE, "the exchange has no RCCL communicator");
  const RcclApi* r = rccl_api();
  ncclResult_t e = r->comm_count(root->nccl_comm, nranks);
  if (e == ncclSuccess) e = r->comm_user_rank(root->nccl_comm, rank);
  if (e != ncclSuccess) return root->fail(DM_E_HIP, std::string("ncclCommCount/UserRank: ") + r->error_string(e));
  return DM_OK;
}

int dm_hier_attach(dm_ctx* leaf, dm_ctx* root, int server, void* const* ring, int nring, void* gathered,
                   void* exchange_stream) {
  DM_ENTER(root);
  if (!leaf || leaf->device != root->device) return root->fail(DM_E_INVAL, "the leaf must share the root's device");
  if (root->hier_G == 0) return root->fail(DM_E_STATE, "set the exchange's layout first (dm_hier_layout)");
  if (server < 0 || server >= root->hier_G) return root->fail(DM_E_RANGE, "server index out of range");
  if (nring < 3 || !ring) return root->fail(DM_E_INVAL, "the publish ring needs at least 3 blocks");
  if (root->hier_G > 1 && !gathered) return root->fail(DM_E_INVAL, "several servers need a gathered buffer");
  int rc = dm_publish_ring(leaf, nring, ring);
  if (rc) return rc;
  if ((rc = dm_hier_pipeline(leaf, leaf->tpl_pipe ? leaf->tpl_lag : 1))) return rc;
  if ((rc = dm_set_stream(root, exchange_stream ? exchange_stream : leaf->stream))) return rc;
  // an exchange on a stream of its own waits for every leaf tick: no stream parts
  if ((rc = set_parts_ok(leaf, root->stream == leaf->stream))) return rc;
  root->hs_leaf = leaf;
  root->hs_server = server;
  root->hs_ring.assign(ring, ring + nring);
  root->hs_gathered = gathered;
  return DM_OK;
}

int dm_hier_step(dm_ctx* leaf, dm_ctx* root, int64_t now_ns) {
  DM_CHECK_CTX(root);
  if (!leaf || root->hs_leaf != leaf) return root->fail(DM_E_STATE, "dm_hier_attach this leaf to the root first");
  int rc = dm_apportion(leaf, now_ns, DM_WRITEBACK | DM_ASYNC | DM_DEFER_JOIN);
  if (rc) return root->fail(rc, "leaf tick: " + leaf->err);  // callers read the root's message
  const int64_t n = (int64_t)root->hs_ring.size();
  void* block = root->hs_ring[(size_t)((leaf->pub_k - 1) % n)];  // what this tick published
  const int G = root->hier_G;
  const void* gathered = block;
  if (G > 1) {
    // the exchange stream after the tick that wrote the block: on the tick's events when
    // its last kernels complete them (no marker on the leaf's queues; the leaf's stream
    // parts stay unjoined), else after a join, on an event
    const bool cover = leaf->stream != root->stream && leaf->tick_covers();
    if (!cover) DM_HIP(root, leaf->join_aux(), "join leaf streams");
    if (leaf->stream != root->stream) leaf->tick_signal_wanted = true;
    if (leaf->stream == root->stream) {
      // stream order
    } else if (cover || (leaf->tick_flagged && leaf->tick_part_mask == 0))
      DM_HIP(root, wait_tick(leaf, leaf->tick_seq, root->stream), "leaf->exchange order");
    else
      DM_HIP(root, leaf->xs_order(dm_ctx::XS_LEAF, leaf->stream, root->stream), "leaf->exchange order");
    const size_t bytes = (size_t)root->hier_stride * 16;
    // (timed as one class on the exchange stream while profiling: bench.py's exchange_us)
    if (root->nccl_comm) {  // every server's block, in server order, over xGMI
      const RcclApi* r = rccl_api();
      ncclResult_t e = ncclSuccess;
      DM_HIP(root, root->timed(KC_HIER_GATHER, root->stream, [&] {
               e = r->all_gather(block, root->hs_gathered, (size_t)root->hier_stride * 2, ncclFloat64,
                                 root->nccl_comm, root->stream);
               return hipSuccess;
             }),
             "gather");
      if (e != ncclSuccess) return root->fail(DM_E_HIP, std::string("ncclAllGather: ") + r->error_string(e));
    } else {  // a rehearsal: this server's slot only
      DM_HIP(root, root->timed(KC_HIER_GATHER, root->stream, [&] {
               return hipMemcpyAsync((char*)root->hs_gathered + (size_t)root->hs_server * bytes, block, bytes,
                                     hipMemcpyDeviceToDevice, root->stream);
             }),
             "gather (local)");
    }
    gathered = root->hs_gathered;
  }
  root->hs_ordered = G > 1;
  rc = dm_hier_root_tick(root, gathered, G, now_ns, leaf, root->hs_server);
  root->hs_ordered = false;
  return rc;
}

int dm_hier_status(dm_ctx* root, uint32_t* status, int n) {
  DM_ENTER(root);
  if (!status || n < 0) return root->fail(DM_E_INVAL, "bad status buffer");
  if (root->hier_servers == 0) return root->fail(DM_E_STATE, "no dm_hier_root_tick yet");
  if (n != root->hier_servers) return root->fail(DM_E_INVAL, "status buffer must hold one word per server");
  DM_HIP(root, download(status, (const uint32_t*)root->hier_status.p, 0, n, root->stream), "hierarchy status");
  DM_HIP(root, hipStreamSynchronize(root->stream), "hierarchy status");
  int bad = 0;
  for (int g = 0; g < n; ++g) bad += status[g] != 0;
  return bad;
}

int dm_set_profiling(dm_ctx* c, int on) {
  DM_CHECK_CTX(c);
  c->profiling = on != 0;
  return DM_OK;
}

int dm_kernel_class_names(const char** names, int max) {
  if (!names && max > 0) return DM_E_INVAL;
  for (int i = 0; i < KC_COUNT && i < max; ++i) names[i] = kClassNames[i];
  return KC_COUNT;
}

int dm_kernel_times(dm_ctx* c, dm_kernel_time* out, int max) {
  DM_ENTER(c);
  DM_HIP(c, hipStreamSynchronize(c->stream), "sync");
  c->collect_profile();
  for (int i = 0; i < KC_COUNT && i < max; ++i) {
    out[i].name = kClassNames[i];
    out[i].launches = c->prof_launches[i];
    out[i].total_ms = c->prof_ms[i];
  }
  return KC_COUNT;
}

int dm_reset_kernel_times(dm_ctx* c) {
  DM_ENTER(c);
  DM_HIP(c, hipStreamSynchronize(c->stream), "sync");
  c->collect_profile();
  for (int i = 0; i < KC_COUNT; ++i) {
    c->prof_ms[i] = 0.0;
    c->prof_launches[i] = 0;
  }
  return DM_OK;
}

int dm_plan_info(dm_ctx* c, int64_t* out, int max) {
  if (!c || !out) return DM_E_INVAL;
  int64_t v[10 + kNumBins];
  v[0] = (int64_t)c->h_tiles.size();
  for (int b = 0; b < kNumBins; ++b) v[1 + b] = (int64_t)c->h_bins[b].size();
  v[1 + kNumBins] = (int64_t)c->h_large.size();
  v[2 + kNumBins] = (int64_t)c->h_chunks.size();
  v[3 + kNumBins] = c->N;
  v[4 + kNumBins] = (c->bin6_wide ? 1 : 0) | (c->bin4_wave ? 2 : 0);  // bit 0: bin 6 on 512 x 8 (else 256 x 16); bit 1: bin 4 on 64 x 16
  v[5 + kNumBins] = c->redo_cap;  // 3/4 of the redo's full-build workgroups the GPU holds at once
  v[6 + kNumBins] = 1;            // every store may speculate (the redo by teams has no bound)
  v[7 + kNumBins] = c->aux_own_queue ? 1 : 0;  // the work classes' streams each have a hardware queue
  int64_t parts = 1;  // the stream parts of the store's one workgroup bin (dm_ctx::kParts), else 1
  for (int b = 0; b < kNumBins; ++b) parts = std::max<int64_t>(parts, c->bin_parts[b]);
  v[8 + kNumBins] = parts;
  // the class streams' queue assignment the calibration chose (dm_ctx::calib): perm[0] +
  // 4 perm[1] + 16 perm[2] + 64 perm[3], or -1 before it has finished (or with shared queues)
  v[9 + kNumBins] = c->calib_best;
  const int n = 10 + kNumBins;
  for (int i = 0; i < n && i < max; ++i) out[i] = v[i];
  return n;
}

int dm_store_lost(dm_ctx* c, int* lost) {
  DM_ENTER(c);
  if (!lost) return c->fail(DM_E_INVAL, "null output");
  (void)c->check_device();  // (records a failure the last sync completed)
  *lost = c->store_lost ? 1 : 0;
  if (c->store_lost) c->err = "internal failure on the device: " + c->lost_msg;
  return DM_OK;
}

int dm_store_stats(dm_ctx* c, int64_t* out, int max) {
  DM_ENTER(c);
  if (!out || max < 0) return c->fail(DM_E_INVAL, "bad output buffer");
  if (!c->store_loaded) return c->fail(DM_E_STATE, "no store loaded");
  std::vector<uint8_t> ex((size_t)c->R);
  DM_HIP(c, download(ex.data(), (const uint8_t*)c->expl.p, 0, c->R, c->stream), "read row states");
  DM_HIP(c, hipStreamSynchronize(c->stream), "read row states");
  int64_t v[4] = {0, 0, 0, 0};
  for (int64_t r = 0; r < c->R; ++r) {
    if (ex[(size_t)r] >= 2) {
      v[0] += 1;
      v[1] += c->h_seg_off[r + 1] - c->h_seg_off[r];
    } else if (ex[(size_t)r] == 1) {
      v[2] += 1;
    }
  }
  v[3] = c->R;
  for (int i = 0; i < 4 && i < max; ++i) out[i] = v[i];
  return 4;
}

}  // extern "C"
