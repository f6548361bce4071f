// dm_device.h — structures shared by the host runtime and the gfx950 kernels.
#pragma once
#include <stdint.h>

namespace dm {

constexpr int64_t kReleased = INT64_MIN;
constexpr int64_t kNs = 1000000000LL;

// Dispatch bins.  A segment of n rows goes to:
//   n <= kSmallMax            : wave-packed literal path (many resources per wave)
//   n <= 64                   : one wave per resource (64x1)
//   n <= 1024                 : one 256-thread workgroup, R = 1, 2, 4 rows per thread in VGPRs
//   n <= 2048 / 4096          : one 512- / 1024-thread workgroup, 4 rows per thread
//   n >  kLargeMin            : multi-workgroup chunks of kChunkRows rows
constexpr int kSmallMax = 16;
constexpr int kLargeMin = 4096;
constexpr int kChunkRows = 4096;
constexpr int kNumBins = 6;  // 64x1, 256x1, 256x2, 256x4, 512x4, 1024x4

struct Pack {  // a run of consecutive small resources covering <= 64 rows
  int32_t first_seg;
  int32_t nseg;  // <= 63
  int64_t row0;
  int32_t nrows;  // <= 64
  int32_t maxlen;  // longest resource in the pack
};

struct WorkItem {  // one resource of a size bin: no dependent load before its rows
  int32_t seg;
  int32_t n;
  int64_t lo;
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
};

struct DevParams {
  const int64_t* seg_off;
  // lease table (SoA).  out_* alias these in writeback mode, so no __restrict__.
  const double* wants;
  const double* has;
  const int64_t* sub;
  const int64_t* expiry;
  // per-resource configuration
  const int32_t* kind;
  const double* capacity;
  const int64_t* lease_len_s;
  const int64_t* refresh_s;
  const int64_t* learning_end;
  const int64_t* parent_expiry;
  const double* safe_cap;
  // store running sums (parity mode input)
  const int64_t* agg_count;
  const double* agg_sum_has;
  const double* agg_sum_wants;
  // lease outputs
  double* out_gets;
  int64_t* out_expiry;
  double* out_wants;  // writeback only: released rows zeroed (else nullptr)
  int64_t* out_sub;   // writeback only
  // per-resource outputs
  int64_t* res_count;
  double* res_sum_has;
  double* res_sum_wants;
  double* res_safe;
  int64_t now;
  int32_t recompute;
  int32_t pad;
};

}  // namespace dm
