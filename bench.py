"""Benchmark: client leases apportioned per second (whole node) + % of HBM peak.

One step = one apportionment tick over every lease of the rank's store: the
device-resident snapshot is decided (Clean, learning mode, the resource's
algorithm) and written back (DM_WRITEBACK), inputs already resident in HBM.
With the hierarchy on (the default for the north-star workload c3), every step
also runs the intermediate-server exchange (publish per-resource totals, one
all-gather over RCCL, the root's apportionment, this server's grants), pipelined
beside the next leaf tick (dm_hier_pipeline).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c1ps|c2|c3|c4] [--hier on|off|auto]
                  [--layout auto|sharded|replicated]

configs[3] (c3, the default): ONE 100M-lease snapshot (100k resources x 1k
clients) sharded by resource id over the N GPUs (hierarchy.partition), each GPU
the intermediate server of its range -- strong scaling, the whole node's leases
per step are 100M at every N.  --layout replicated gives every GPU its own
full-size store instead (weak scaling; reported under extra.weak_scaling at N > 1).

--gpus N > 1 without a torch.distributed environment starts N ranks itself
(python -m torch.distributed.run, one process per GPU, started before this
process touches the GPU) and exits with their status.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_COPY_CEIL_GBS = 6290.0  # measured float4 copy ceiling (same table)
METRIC = "client leases apportioned/sec (whole node) + % HBM peak, FairShare, 1-8 GPU"
DEFAULT_WORKLOAD = "c3"

WORKLOADS = {
    "c1": "C1 (BASELINE configs[1]): 10,000 resources x 1,000 clients per GPU (10M leases), FairShare, uniform wants",
    "c1ps": "C1 (BASELINE configs[1]): 10,000 resources x 1,000 clients per GPU (10M leases), ProportionalShare",
    "c2": "C2 (BASELINE configs[2]): 1M resources, Zipf 1..1M clients (13,970,034 leases), mixed kinds, 5% learning",
    "c3": "C3 (BASELINE configs[3], north-star size): 100,000 resources x 1,000 clients = 100M leases, FairShare",
    "c4": "C4 (BASELINE configs[4]) per GPU: 125M-lease device-resident store (1B over 8 GPUs), 125k resources x "
          "1k client slots, FS/PS mixed, 5% learning; every step = 5 s refresh tick: 10% wants updates and 1% "
          "departures + 1% new clients (narrow 20-B arrival records) over PCIe, then the tick",
}


C3_R, C3_CLIENTS = 100_000, 1_000


def c3_bounds(world: int):
    """configs[3]: the resource-id ranges of the node's GPUs (contiguous, balanced by
    lease count: hierarchy.partition)."""
    from doorman_amd.hierarchy import partition
    return partition(np.full(C3_R, C3_CLIENTS), world)


def c2_bounds(world: int, snap=None):
    """configs[2] over N GPUs: contiguous resource-id ranges of the one Zipf snapshot,
    balanced by predicted tick cost (hierarchy.tick_cost: bytes per lease and per
    resource), not by lease count -- a lease-count split leaves the 500k singletons'
    97-B records on the last shard (2.2x the mean bytes at N = 8)."""
    from doorman_amd import workloads as W
    from doorman_amd.hierarchy import partition, tick_time
    sizes = np.diff(snap["seg_off"]) if snap is not None else W.zipf_sizes()
    return partition(sizes, world, tick_time(sizes))


C2_PARTITIONS = ("classes", "lpt", "contiguous")
_OWNERS = {}


def c2_shard_ids(world: int, rank: int, partition: str = "classes", snap=None) -> np.ndarray:
    """configs[2]'s resource ids of one rank: classes (default) -- hierarchy.assign_by_class,
    every rank 1/N of every size class and the mean bytes; lpt -- hierarchy.assign_lpt
    over all resources at once; contiguous -- c2_bounds' range."""
    from doorman_amd import workloads as W
    from doorman_amd.hierarchy import assign_by_class, assign_lpt
    sizes = np.diff(snap["seg_off"]) if snap is not None else W.zipf_sizes()
    if partition == "contiguous":
        b = c2_bounds(world, snap)
        return np.arange(int(b[rank]), int(b[rank + 1]), dtype=np.int64)
    key = (partition, world, len(sizes), int(sizes.sum()))
    if key not in _OWNERS:
        _OWNERS[key] = (assign_lpt if partition == "lpt" else assign_by_class)(sizes, world)
    return np.flatnonzero(_OWNERS[key] == rank).astype(np.int64)


def make_workload(name: str, rank: int, world: int = 1, layout: str = "replicated", partition: str = "classes"):
    from doorman_amd import workloads as W
    if name == "c1":
        return W.c1(seed=1 + 1000 * rank, kind=W.FAIR_SHARE)
    if name == "c1ps":
        return W.c1(seed=1 + 1000 * rank, kind=W.PROPORTIONAL_SHARE)
    if name == "c2":
        if layout == "sharded":  # this rank's resources of the one 1M-resource Zipf snapshot
            snap = W.c2(seed=2)
            if world <= 1:
                return snap
            if partition == "contiguous":
                b = c2_bounds(world, snap)
                return W.subset_range(snap, int(b[rank]), int(b[rank + 1]))
            return W.subset(snap, c2_shard_ids(world, rank, partition, snap))
        return W.c2(seed=2 + 1000 * rank)
    if name == "c3":
        if layout == "sharded":  # this rank's range of the one 100M-lease snapshot
            b = c3_bounds(world)
            return W.uniform_range(C3_R, C3_CLIENTS, int(b[rank]), int(b[rank + 1]), kind=W.FAIR_SHARE, seed=3)
        return W.uniform_range(C3_R, C3_CLIENTS, 0, C3_R, kind=W.FAIR_SHARE, seed=3 + 1000 * rank)
    if name == "c4":
        snap = W.uniform(125_000, 1_000, kind="mixed", seed=4 + 1000 * rank)
        rng = np.random.default_rng(40 + rank)
        R = len(snap["seg_off"]) - 1
        snap["learning_end_ns"] = np.where(rng.random(R) < 0.05, W.NOW_NS + 3600 * W.NS,
                                           W.INT64_MIN).astype(np.int64)
        free = rng.random(len(snap["wants"])) < 0.02  # slack slots for new clients
        snap["wants"][free] = 0.0
        snap["has"][free] = 0.0
        snap["subclients"] = np.where(free, 0, 1).astype(np.int64)
        snap["expiry_ns"][free] = W.RELEASED
        snap["expiry_ns"][~free] = W.NOW_NS + 3600 * W.NS
        return W.add_store_sums(snap)
    raise SystemExit(f"unknown workload {name}")


# A writeback tick (every bench step) reads wants 8 + has 8 + subclients 4 and writes
# gets 8 per lease: the leases it grants follow their resource's expiry, so no 8-B
# expiry is read or written per lease.  SURVEY.md section 8(d)'s
# canonical layout moves 48 B (int64 subclients, expiry read and written per lease).
LEASE_BYTES = 28
DENSE_LEASE_BYTES = 24  # a dense resource's rows (one subclient count, every row a live follower): no subclients read
SURVEY_LEASE_BYTES = 48
RESOURCE_BYTES = 97  # config 32 B + running sums and follower expiry 32 B read and written + explicit flag 1 B


def algorithmic_bytes(n_leases: int, n_resources: int, dense_leases: float = 0) -> int:
    """Bytes a writeback tick must move with this store layout: per lease read wants,
    has, subclients (int32: the boundary restricts them to [0, 2^31 - 1)), write gets
    -- without the subclients read for the rows of dense resources (dm_store_stats);
    per resource the config record and the running sums in and out.  Re-reads are
    not counted."""
    return int(round(LEASE_BYTES * n_leases - (LEASE_BYTES - DENSE_LEASE_BYTES) * dense_leases
                     + RESOURCE_BYTES * n_resources))


L3_BYTES = 256 << 20    # MI355X Infinity Cache (MALL), MI355X_MICROARCH.md chip-level parameters
STREAM_BYTES = 1 << 30  # dm_device.h kStreamBytes: a store with 48 * N above it writes gets to an alternate column


def tick_footprint_bytes(snap, dense_leases: float = 0.0) -> dict:
    """Distinct bytes one writeback tick touches (each line once, reads and writes of the
    same line together): wants, has, the subclients column except for dense rows, the
    alternate gets column when the tick writes one (dm_runtime.cpp: a store with 48 * N >
    kStreamBytes, or one with a > 4096-row resource, whose speculative chain writes gets
    before they are verified), and per resource the 32-B config, 32-B sums and state byte.
    At or below the 256 MiB Infinity Cache the tick's lines stay cache-resident from tick
    to tick, so the rocprof FETCH_SIZE / WRITE_SIZE counts (which include Infinity-Cache
    hits, MI355X_MICROARCH.md HBM/rocprofv3 section) and any GB/s over these bytes
    measure cache bandwidth, not HBM."""
    sizes = np.diff(snap["seg_off"])
    N, R = int(sizes.sum()), len(sizes)
    alternate = 48 * N > STREAM_BYTES or bool((sizes > 4096).any())
    b = 16 * N + 4 * (N - dense_leases) + (8 * N if alternate else 0) + 65 * R
    return {"tick_footprint_bytes": int(round(b)), "alternate_gets_column": alternate,
            "l3_resident": bool(b <= L3_BYTES)}


def dense_fraction(eng, snap) -> float:
    """Share of the rows of resources with 257..4096 rows (the workgroup kernels,
    the only ones that keep the dense state) that sit in dense resources, in the
    store's state right now (dm_store_stats)."""
    sizes = np.diff(snap["seg_off"])
    group = int(sizes[(sizes >= 257) & (sizes <= 4096)].sum())
    return eng.store_stats()["dense_leases"] / group if group else 0.0


SMALL_MAX = 4  # dm_device.h kSmallMax: resources of at most this many rows run in the tiles
# the sub-wave bins by row range (their names are the library's bin names; each runs in
# several G x R shapes inside the one k_subs launch, dm_device.h SubBins)
_SUB_EDGES = [("sub8x2", 5, 16), ("sub16x2", 17, 32), ("sub16x4", 33, 64), ("sub32x4", 65, 128),
              ("wave64x4", 129, 256)]
_GROUP_EDGES = [("block128x4", 257, 512), ("block128x8", 513, 1024), ("block256x8", 1025, 2048),
                ("block2k4k", 2049, 4096)]
# the kernel classes that read 24 B per lease of a dense resource (no subclients column):
# the 128-thread mixed kernels (they load by the hint) and every dense kernel of the split form
DENSE_READERS = ("block128x4", "block128x8") + tuple(n + "_dense" for n, _, _ in _GROUP_EDGES)


def kernel_units(snap):
    """(leases, resources) each kernel class that dm_kernel_times can report processes
    per launch (tests/test_bench_model.py checks the names against the library's).
    Classes that move no lease rows of their own carry (0, resources) or (0, 0)."""
    sizes = np.diff(snap["seg_off"])
    R = len(sizes)
    units = {}

    def rng(lo, hi):
        m = (sizes >= lo) & (sizes <= hi)
        return int(sizes[m].sum()), int(m.sum())
    small = sizes <= SMALL_MAX
    units["small_tiles"] = (int(sizes[small].sum()), int(small.sum()))
    for name, lo, hi in _SUB_EDGES + _GROUP_EDGES:
        units[name] = rng(lo, hi)
    units["subs_merged"] = rng(SMALL_MAX + 1, 256)  # the sub-wave bins in one launch (k_subs)
    for name, _, _ in _GROUP_EDGES:  # the split form's two kernels
        units[name + "_dense"] = units[name]
        units[name + "_rest"] = (0, 0)  # only what the dense kernel queued; counted with the dense kernel
    big = rng(4097, 1 << 62)
    # the chain's launches, the speculative chain (one pass over every large lease), the
    # heterogeneous chain's launches: each over every row of the > 4096-row class
    for name in ("large_a", "large_b", "large_c", "large_map", "large_fin", "large_spec", "large_t",
                 "large_c_het", "large_e", "large_map_het"):
        units[name] = big
    # the redo rewrites only the resources whose speculation failed (none in a steady tick:
    # its launch then reads one word per workgroup)
    units["large_redo"] = (0, 0)
    units["general"] = rng(SMALL_MAX + 1, 1 << 62)  # heterogeneous FairShare: any resource above the tiles may land there
    units["hier_publish"] = (0, R)
    units["hier_root"] = (0, R)
    units["hier_gather"] = (0, 0)  # 16 B per resource per server: a collective, not HBM streaming
    units["store_upsert"] = units["store_release"] = units["decide"] = (0, 0)  # not on a tick
    return units


def kernel_lease_bytes(name, leases_k, dense_frac):
    """Algorithmic bytes per launch of one kernel class, split as (28-B leases, 24-B leases).
    large_spec: a steady writeback tick through the chain reads no subclients column
    (the last tick's live bits and per-chunk counts): 24 B per lease."""
    if name == "large_spec":
        return leases_k
    if name in DENSE_READERS:
        return dense_frac * leases_k
    return 0.0


def streaming_step(eng, snap, rank, n_ticks, asynchronous=True):
    """configs[4]: one 5 s refresh tick of a device-resident store.  Per tick the
    host sends 10% wants updates (row mask + packed values, narrow Assign), releases
    1% of the clients (departures, store.go:142-151), inserts 1% new clients into
    free slots (upsert onto released rows) -- all three in one store batch --
    then the tick runs with writeback.  The update batches (what the RPCs would deliver) are generated
    before the timed region.  asynchronous (the default): the batch through
    dm_store_apply_async, so one round's PCIe copies follow the previous round's back to
    back (the host waits only for the batch two rounds back); step.finish retires the
    batches in flight (a rejected one raises)."""
    from doorman_amd import workloads as W
    rng = np.random.default_rng(400 + rank)
    N = len(snap["wants"])
    alive = snap["expiry_ns"] != W.RELEASED
    pool = np.flatnonzero(~alive)
    now = W.NOW_NS
    batches = []
    for _ in range(n_ticks):
        off = int(rng.integers(0, 10))
        upd = np.arange(off, N, 10, dtype=np.int64)
        upd = upd[alive[upd]]
        off = int(rng.integers(0, 100))
        gone = np.arange(off, N, 100, dtype=np.int64)
        gone = gone[alive[gone]]
        new = np.sort(pool[: len(gone)])
        pool = np.concatenate([pool[len(gone):], gone])
        alive[gone] = False
        alive[new] = True
        now += 5 * W.NS
        k = len(new)
        # the wants refresh crosses PCIe as a row mask + packed values (1.25 B of mask
        # per update at 10% instead of an 8-B row index: dm_store_update_wants_mask);
        # arrivals as narrow records: row, wants, int32 subclients (has 0 and the
        # expiry now + lease length implied: the Assign of a new client, store.go:153-167)
        cols = (W.rows_to_mask(upd, N), rng.uniform(0.5, 1.5, len(upd)), gone, new, rng.uniform(0.5, 1.5, k),
                np.ones(k, np.int32))
        # the RPC layer would decode requests straight into page-locked buffers
        # (dm_host_alloc), which then cross PCIe by DMA
        pinned = []
        for a in cols:
            h = eng.host_empty(len(a), a.dtype)
            h[:] = a
            pinned.append(h)
        batches.append((*pinned, now))
    it = iter(batches)

    def apply_only():
        mask, w, gone, new, nw, ns, t = next(it)
        # the round's three update kinds, one call
        eng.apply(mask, w, gone, (new, None, nw, ns, None), now_ns=t, asynchronous=asynchronous)
        step.last_now = t  # (busy_kernel_probe ticks on at the last applied round's time)
        return t

    def step():
        eng.apportion(apply_only(), writeback=True, asynchronous=True)

    step.last_now = now
    step.apply_only = apply_only
    step.finish = eng.apply_wait if asynchronous else (lambda: None)  # the state a tick starts from (bench's dense share at tick time)
    return step


# ---------------------------------------------------------------------------
# CPU baseline: the reference's algorithm restated in C
# (oracle/, test infrastructure), timed on this host's cores.
# ---------------------------------------------------------------------------
def host_cores():
    """CPUs this process may actually use: the scheduler affinity, capped by the
    cgroup CPU quota (a GPU box grants one GPU's share of a large host) and by
    OMP_NUM_THREADS when the environment sets it (the box does: its CPU share)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    n = usable
    if quota:
        n = min(n, quota)
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n), {"usable_cores": usable, "cgroup_cpu_quota": quota, "omp_num_threads": env}


def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count()}


def subset_rows(snap, max_rows):
    """the leading resources of a snapshot holding at most max_rows leases"""
    from doorman_amd import workloads as W
    so = snap["seg_off"]
    k = int(np.searchsorted(so, max_rows, side="right")) - 1
    return W.subset(snap, np.arange(max(k, 1)))


def cpu_baseline(snap, now_ns, budget_s=12.0):
    """The reference algorithm restated in C, timed on a bounded sample of this
    workload at the host's width:
      value          literal per-request Resource.Decide on a private store copy (O(n) per
                     request, as the reference), OpenMP pool over resources;
      closed_form_mt the closed form (same outputs) over all resources;
      configs0       BASELINE configs[0] (1 resource x 1,000 clients, ProportionalShare)."""
    from doorman_amd import workloads as W
    from oracle import oracle as O
    threads, cores = host_cores()
    so = snap["seg_off"]
    sizes = np.diff(so)
    rng = np.random.default_rng(0)
    cand = rng.permutation(np.flatnonzero(sizes > 0))
    row_cap = 4000  # O(n^2) per resource: a slice of clients of the giant resources
    gets = np.empty(len(snap["wants"]))
    # calibrate on a small batch, then one batch sized to the budget
    k0 = min(len(cand), 4 * threads)
    t0 = time.perf_counter()
    O.apportion_literal_sample(snap, cand[:k0], row_cap, now_ns, gets, threads)
    t_cal = time.perf_counter() - t0
    k1 = int(min(len(cand) - k0, max(threads, k0 * max(budget_s - t_cal, 0.0) / max(t_cal, 1e-3))))
    t0 = time.perf_counter()
    rows = O.apportion_literal_sample(snap, cand[k0:k0 + k1], row_cap, now_ns, gets, threads) if k1 > 0 else 0
    t_lit = time.perf_counter() - t0
    if k1 <= 0:
        rows, t_lit, k1 = O.apportion_literal_sample(snap, cand[:k0], row_cap, now_ns, gets, threads), t_cal, k0
    # the closed form over the whole snapshot
    O.apportion(subset_rows(snap, 2000), now_ns, "closed", threads=threads)  # warm the pool
    reps, t_mt = 0, 0.0
    while reps < 3 and t_mt < 5.0:
        t0 = time.perf_counter()
        O.apportion(snap, now_ns, "closed", threads=threads)
        t_mt += time.perf_counter() - t0
        reps += 1
    # configs[0]: the reference's own CPU case, single resource (one thread: one store)
    c0 = W.c0()
    n0 = len(c0["wants"])
    g0 = np.empty(n0)
    reps0, t0s = 0, 0.0
    while t0s < 1.0:
        t0 = time.perf_counter()
        O.apportion_literal_rows(c0, 0, 0, n0, now_ns, g0)
        t0s += time.perf_counter() - t0
        reps0 += 1
    return {
        "value": rows / t_lit if t_lit > 0 else None,
        "unit": "leases/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{rows} leases of {k1} resources of the same workload (first {row_cap} clients of each), every "
                  f"one decided by the literal C restatement of Resource.Decide (go/server/doorman/resource.go:100-113) "
                  f"on a private store copy (O(n) per request as in the reference), OpenMP pool over resources on "
                  f"{threads} threads, {t_lit:.1f} s",
        "closed_form_mt": {
            "value": reps * len(snap["wants"]) / t_mt,
            "unit": "leases/s",
            "cores": threads,
            "sample": f"whole snapshot x{reps}: oracle/ closed form (SURVEY.md §8a), OpenMP over resources",
        },
        "configs0": {
            "value": reps0 * n0 / t0s,
            "unit": "leases/s",
            "cores": 1,
            "kind": "port",
            "sample": f"BASELINE configs[0]: 1 resource x {n0} clients, ProportionalShare (workloads.c0), literal "
                      f"per-request Decide x{reps0}, one thread (one store)",
        },
        "host": {**host_info(), **cores, "threads_used": threads},
    }


# ---------------------------------------------------------------------------
# timing
# ---------------------------------------------------------------------------
def timed_steps(torch, eng, step, steps, warmup, sync_ranks, extra_warm=True, also=()):
    """W untimed warm-up steps, then more until ~0.3 s of ticks have run (the first
    milliseconds of back-to-back ticks run ~10% slow: C3 measured 843 us/tick after 3
    warm-up ticks, 765 after 30; the count is agreed over ranks), then K timed steps
    between barrier + synchronize, then K profiled steps (HIP events around every
    launch, on the stream each kernel runs on)."""
    t_w = time.perf_counter()
    for _ in range(max(warmup, 1)):
        step()
    eng.sync()
    per_step = (time.perf_counter() - t_w) / max(warmup, 1)
    extra = min(20000, int(0.3 / max(per_step, 1e-6))) if extra_warm else 0
    extra = sync_ranks("max_int", extra)
    for i in range(extra):
        step()
        if i % 8 == 7:
            eng.sync()
    eng.sync()
    ext = torch.cuda.ExternalStream(eng.stream)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sync_ranks("barrier", None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(ext)
    for _ in range(steps):
        step()
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps (the GPU runs behind it)
    eng.join()  # every class stream's work before the closing event
    ev1.record(ext)
    eng.sync()
    torch.cuda.synchronize()
    sync_ranks("barrier", None)
    elapsed = time.perf_counter() - t0
    stream_ms = ev0.elapsed_time(ev1)
    prof = [eng] + list(also)  # the exchange's root round runs on the root engine
    for e in prof:
        e.set_profiling(True)
        e.reset_kernel_times()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ktimes = {}
    for e in prof:
        e.sync()
        ktimes.update(e.kernel_times())
        e.set_profiling(False)
    return {"elapsed": elapsed, "stream_ms": stream_ms, "ktimes": ktimes, "warm_run": max(warmup, 1) + extra,
            "host_enqueue_s": t_enq}


def roofline_of(workload, snap, run, steps, single_kernel_tick):
    """Roofline object for the dominant kernel (largest share of in-stream time)."""
    ktimes = run["ktimes"]
    if not ktimes:
        return None
    name, (launches, total_ms) = max(ktimes.items(), key=lambda kv: kv[1][1])
    avg_s = total_ms / launches / 1e3
    single = single_kernel_tick and len(ktimes) == 1 and launches == steps
    # stream parts (dm_plan_info): the store's one workgroup bin runs as `parts` concurrent
    # launches over its halves, unjoined from tick to tick; its roofline is the whole bin's
    # bytes per tick over the tick's time (both launches together), not one half over a
    # launch that shares the GPU with the other
    parts = int(run.get("parts", 1))
    in_parts = parts > 1 and len(ktimes) == 1 and launches == parts * steps
    if single or in_parts:  # one kernel class per tick: HIP events around the timed region itself
        avg_s = run["stream_ms"] / steps / 1e3
    units = kernel_units(snap)
    if name not in units:
        raise KeyError(f"bench.kernel_units has no entry for kernel class {name!r}: its bytes per launch are unknown")
    leases_k, res_k = units[name]
    dense_k = kernel_lease_bytes(name, leases_k, run.get("dense_frac", 0.0))
    alg = algorithmic_bytes(leases_k, res_k, dense_k)
    achieved = alg / avg_s / 1e9
    fp = tick_footprint_bytes(snap, tick_dense_leases(snap, run.get("dense_frac", 0.0)))
    l3 = fp["l3_resident"]
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get(name, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
        if traffic is not None and in_parts:  # the PMC passes count per launch: per tick, both parts
            traffic = traffic * parts
    return {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            # a cache-resident tick (footprint <= 256 MiB) is not HBM evidence: no HBM fraction
            "frac": None if l3 else round(achieved / HBM_PEAK_GBS, 4),
            "frac_of_copy_ceiling": None if l3 else round(achieved / HBM_COPY_CEIL_GBS, 4),
            **fp,
            "frac_l3": round(achieved / HBM_PEAK_GBS, 4) if l3 else None,
            "l3_note": ("the tick's distinct bytes fit the 256 MiB Infinity Cache: they stay cache-resident from "
                        "tick to tick, so achieved and the PMC traffic (FETCH_SIZE counts Infinity-Cache hits) "
                        "measure cache bandwidth; frac_l3 is achieved over the HBM spec for comparison only"
                        if l3 else None),
            "traffic": traffic,
            "traffic_source": f"profiles/pmc_{workload}.json (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, calibrated)",
            "algorithmic_bytes_per_launch": alg,
            "leases_per_launch": leases_k, "resources_per_launch": res_k,
            "bytes_model": (f"{LEASE_BYTES} B per lease (read wants, has, int32 subclients; write gets: granted "
                            f"leases follow their resource's expiry), {DENSE_LEASE_BYTES} B for the rows of dense "
                            f"resources (every row a live follower with one subclient count: no subclients read) "
                            f"and for large_spec's rows (a steady tick through the chain: the last tick's live "
                            f"bits instead of the subclients column) + {RESOURCE_BYTES} B per resource; the "
                            f"canonical layout of SURVEY.md 8(d) moves {SURVEY_LEASE_BYTES} B per lease"),
            "dense_lease_share": round(dense_k / leases_k, 4) if leases_k else 0.0,
            "survey_layout_equivalent_GBs": round((SURVEY_LEASE_BYTES * leases_k + 64 * res_k) / avg_s / 1e9, 1),
            # SURVEY.md 8(d) / BASELINE.md 3's canonical 48 B x N + 64 B x R over the same launch time:
            # above 1 here because this layout does not move those bytes (layout_note)
            "frac_survey_model": round((SURVEY_LEASE_BYTES * leases_k + 64 * res_k) / avg_s / 1e9 / HBM_PEAK_GBS, 4),
            "layout_note": ("frac is over the bytes this layout must move: a lease granted by a writeback tick "
                            "follows its resource's expiry (one follow_exp per resource, no 8-B expiry read or "
                            "written per lease) and subclients are int32 (28 B per lease); a dense resource's rows "
                            "(every row a live follower with one count, recorded in its state byte) skip the "
                            "subclients column (24 B).  PMC traffic (traffic) confirms the kernel moves these "
                            "bytes, not the canonical 48 (frac_survey_model)"),
            "avg_launch_us": round(avg_s * 1e6, 2),
            "kernel_time_share": round(total_ms / sum(v[1] for v in ktimes.values()), 3),
            "kernel_time_share_note": "of the summed event time of every profiled kernel class of a step (the "
                                      "exchange's publish and root round included; concurrent classes overlap)",
            "timed_region_stream_us_per_step": round(run["stream_ms"] * 1e3 / steps, 2),
            "duration_source": ("HIP event pair around the timed region on the kernel's stream (one kernel "
                                "per tick)" if single else
                                f"HIP event pair around the timed region (the bin's {parts} concurrent stream-part "
                                f"launches per tick, joined at its end; bytes and traffic per tick)" if in_parts else
                                "HIP events around every launch, profiled region"),
            "stream_parts": parts}


# ---------------------------------------------------------------------------
# exchange self-check (N > 1 runs: the RCCL leg of the exchange checks itself)
# ---------------------------------------------------------------------------
def _minF(l, r):
    return r if l > r else l  # algorithm.go:50-55


def root_round_one(now, cfg, row, sums, flags, sum_wants, count):
    """The root's round for one resource of the sharded layout (one root row, its
    owner's; k_hier_tick with K = 1), restated for the bench's self-check from
    server.go:822-901 -> resource.go:100-113 -> algorithm.go:95-302 / store.go:153-181:
    Clean, then the owner's request (SumWants, Count) decided by the resource's
    algorithm against the cleaned store, then the owner's new template
    (server.go:279-313).  Returns (template fields, gets) or None for a rejected block."""
    f64 = np.float64
    kind, cap, lease_s, refresh_s, learn_end, parent, safe = cfg
    if flags != 0:
        return None
    w, h, sub, e = f64(row[0]), f64(row[1]), int(row[2]), int(row[3])
    cnt, sh, sw = int(sums[0]), f64(sums[1]), f64(sums[2])
    released = e == W_RELEASED
    expired = not released and now > e
    live = not released and not expired
    if expired:  # Clean (store.go:169-181)
        sw, sh, cnt = sw - w, sh - h, cnt - sub
    if not live:
        w, h, sub = f64(0.0), f64(0.0), 0
    req = sum_wants > 0.0
    rw, rs = f64(sum_wants), int(count) if sum_wants > 0.0 else 0
    C = f64(0.0) if parent < now else f64(cap)
    learning = learn_end > now
    gets = f64(0.0)
    with np.errstate(all="ignore"):
        if req:
            if learning:
                gets = f64(0.0)  # Learn: the request's Has (an intermediate never fills it)
            elif kind == 0:
                gets = rw
            elif kind == 1:
                gets = _minF(C, rw)
            elif kind == 2:  # ProportionalShare (algorithm.go:213-293)
                eq = C / f64(cnt + (0 if live else rs))
                ds = eq * f64(rs)
                avail = C - sh + h
                if sw <= C or rw <= ds:
                    gets = _minF(rw, avail)
                else:  # the Map: only the requesting row, with its request values, if present
                    x = y = f64(0.0)
                    if live:
                        esp = eq * f64(rs)
                        if rw < esp:
                            x += esp - rw
                        else:
                            y += rw - esp
                    gets = _minF(ds + (rw - ds) * (x / y), avail)
            else:  # FairShare (algorithm.go:95-206): no other row, so round 1 and 2 sum nothing
                avail = C - sh + h
                eq = C / f64(cnt - sub + rs)
                ds = eq * f64(rs)
                if rw <= ds:
                    gets = _minF(rw, avail)
                else:
                    dE = (f64(0.0) / f64(rs)) * f64(rs)
                    if rw < ds + dE:
                        gets = _minF(rw, avail)
                    else:
                        gets = _minF(ds + dE + (f64(0.0) / f64(rs)) * f64(rs), avail)
    if req:
        exp_new = now + int(lease_s) * 1_000_000_000
        sec = exp_new // 1_000_000_000  # time.Unix(sec, 0)
        tpl = (int(kind), float(gets), int(lease_s), int(refresh_s), sec * 1_000_000_000,
               0.0 if np.isnan(safe) else float(safe))
    else:  # the "*" default template (server.go:53-63)
        tpl = (3, 0.0, 20, 1, W_INT64_MAX, 0.0)
    return tpl, float(gets)


W_RELEASED = np.iinfo(np.int64).min
W_INT64_MAX = np.iinfo(np.int64).max
_TPL_FIELDS = ("kind", "capacity", "lease_length_s", "refresh_interval_s", "parent_expiry_ns", "safe_capacity")


def exchange_self_check(torch, dist, ht, leaf, root, bounds, rank, world, g, now, red_dev, corrupt=False,
                        n_sample=64):
    """One more exchange step after the timed ones, then checks that the exchange moved
    the right bytes (for N > 1: the RCCL all-gather's first use in a run):
      blocks  every rank's gathered buffer hashes alike (all-reduce MIN == MAX);
      own     this rank's block sits at its slot of the gathered buffer, and holds its
              leaf's running {SumWants, Count};
      root    rank 0 recomputes, from ITS gathered copy, the root round of a sample of
              every rank's resources (first, last and random ones: the root rows and
              sums before the step, gathered from their owners) and compares the
              templates the owners' leaves took, bit for bit.
    corrupt (test-only): rank world-1 perturbs its gathered copy after the all-gather."""
    import hashlib
    from doorman_amd import _lib
    ht.sync()
    lo, hi = int(bounds[g]), int(bounds[g + 1])
    n = hi - lo
    pre = root.read_store(lo, n)
    pres = root.resources(lo, n, safe=False)
    rng = np.random.default_rng(1234 + g)
    pick = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, max(0, n_sample - 2))])) if n else []
    # the block an exchange publishes: the leaf's sums after this step's tick (pipelined:
    # the tick writes it) or before it (unpipelined: published first)
    lr = None if ht.pipelined else leaf.resources(safe=False)
    gather0 = ht.gather
    if corrupt and rank == world - 1:
        def bad(src, dst):
            gather0(src, dst)
            dst[1, 0] += 1.0  # block 0's first SumWants
        ht.gather = bad
    try:
        ht.tick(now)
        ht.sync()
    finally:
        ht.gather = gather0
    k = (ht.step - 1) % len(ht.totals)
    if corrupt and rank == world - 1 and ht.native is not None:  # (the library gathered it: corrupt the copy)
        ht.gathered[k][1, 0] += 1.0
        torch.cuda.synchronize()
    gathered = ht.gathered[k].cpu().numpy().copy()
    S = ht.stride
    own = ht.totals[k].cpu().numpy()
    own_ok = gathered[g * S:(g + 1) * S].tobytes() == own.tobytes()
    lr = lr or leaf.resources(safe=False)
    pub_ok = (np.ascontiguousarray(own[1:1 + n, 0]).tobytes() == lr["sum_wants"].tobytes()
              and np.ascontiguousarray(own[1:1 + n, 1]).view(np.int64).tobytes()
              == lr["count"].astype(np.int64).tobytes())
    if ht.pipelined:  # take the staged templates of this exchange
        _lib.check(leaf._L.dm_hier_pipeline(leaf._ctx, 0), leaf._ctx, leaf._L)
        _lib.check(leaf._L.dm_hier_pipeline(leaf._ctx, ht.lag), leaf._ctx, leaf._L)
    tpl = leaf.config()
    samples = [(lo + int(i), (pre["wants"][i], pre["has"][i], int(pre["subclients"][i]), int(pre["expiry_ns"][i])),
                (int(pres["count"][i]), pres["sum_has"][i], pres["sum_wants"][i]),
                tuple(tpl[f][i].item() for f in _TPL_FIELDS)) for i in pick]
    h = int.from_bytes(hashlib.blake2b(gathered.tobytes(), digest_size=8).digest(), "little", signed=True)
    ok = 1 if (own_ok and pub_ok) else 0
    if world > 1:
        allsamp = [None] * world
        dist.all_gather_object(allsamp, samples)
        allsamp = [x for part in allsamp for x in part]
        t = torch.tensor([h, -h, ok], dtype=torch.int64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        hmin, hmax, ok_all = int(t[0].item()), -int(t[1].item()), int(t[2].item())
    else:
        allsamp, hmin, hmax, ok_all = samples, h, h, ok
    if rank != 0:
        return None
    rc = root.config()
    cfg_cols = [rc[f] for f in ("kind", "capacity", "lease_length_s", "refresh_interval_s", "learning_end_ns",
                                "parent_expiry_ns", "safe_capacity")]
    owners = np.searchsorted(bounds, [r for r, *_ in allsamp], side="right") - 1
    mism, rejected = 0, 0
    for (r, row, sums, got), o in zip(allsamp, owners):
        blk = gathered[o * S:(o + 1) * S]
        f = int(blk[0, 0:1].view(np.uint64)[0])
        flags = (f & 0xFFFFFFFF) | (f >> 32)  # record 0's two flags words (one per stream part)
        v = blk[1 + r - int(bounds[o])]
        res = root_round_one(now, [c[r] for c in cfg_cols], row, sums, flags, v[0], int(v[1:2].view(np.int64)[0]))
        if res is None:
            rejected += 1
            continue
        want = res[0]
        if any(np.float64(a).tobytes() != np.float64(b).tobytes() if isinstance(a, float) else a != b
               for a, b in zip(want, got)):
            mism += 1
    return {"consistent": bool(hmin == hmax and ok_all == 1 and mism == 0 and rejected == 0),
            "blocks_hash_equal": hmin == hmax, "own_blocks_ok": ok_all == 1,
            "sample": len(allsamp), "template_mismatches": mism, "rejected": rejected,
            "corrupted_on_purpose": bool(corrupt),
            "how": "one more exchange step after the timed ones: gathered buffers hashed and compared over ranks "
                   "(all-reduce MIN/MAX), every rank's own block at its slot and equal to its leaf's running sums, "
                   "and rank 0 recomputing from its gathered copy the root round of a sample of every rank's "
                   "resources and comparing the owners' templates bit for bit"}


def tick_dense_fraction(eng, snap, step) -> float:
    """The dense share of the workgroup bins' rows in the state a tick starts from: after
    a writeback tick for back-to-back ticks; for configs[4] after a round's store updates
    (step.apply_only), which leave most resources with explicit rows, not dense."""
    if hasattr(step, "apply_only"):
        step.apply_only()
        eng.sync()
    return dense_fraction(eng, snap)


def tick_dense_leases(snap, dense_frac) -> float:
    """Rows of dense resources in a tick: dense_frac of the workgroup bins' rows."""
    sizes = np.diff(snap["seg_off"])
    return dense_frac * int(sizes[(sizes >= 257) & (sizes <= 4096)].sum())


def tick_fracs(snap, dense_frac, t_step) -> dict:
    """The tick's algorithmic bytes over its step time against the HBM spec -- null for a
    cache-resident tick (tick_footprint_bytes), whose rate goes to tick_frac_l3."""
    R, N = len(snap["seg_off"]) - 1, int(snap["seg_off"][-1])
    dense = tick_dense_leases(snap, dense_frac)
    tick_bytes = algorithmic_bytes(N, R, dense)
    f = round(tick_bytes / t_step / 1e9 / HBM_PEAK_GBS, 4)
    fp = tick_footprint_bytes(snap, dense)
    return {"tick_hbm_frac": None if fp["l3_resident"] else f, "tick_frac_l3": f if fp["l3_resident"] else None,
            "tick_algorithmic_bytes": tick_bytes, **fp}


def busy_kernel_probe(eng, snap, now, dense_frac, ticks=20, warm_s=0.3):
    """configs[4]'s tick kernel with the GPU kept busy: after the timed streaming
    rounds, the same store ticked back to back at the last round's time with no
    update between (~0.3 s first, as timed_steps' warm-up), HIP events around every
    launch.  The same kernel on the same store runs 15-20 % faster after sustained
    back-to-back ticks than inside the streaming step (tools/c4_variants.py: C3's
    kernel after 4 ticks 516 us, after 0.3 s 416 us on one box; a ramp only sustained
    memory load reaches: profiles/r06_c4_variants.md).  Reported beside the step's own
    roofline, never in its place."""
    t_w = time.perf_counter()
    n = 0
    while time.perf_counter() - t_w < warm_s:
        eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
        n += 1
        if n % 8 == 0:
            eng.sync()
    eng.sync()
    eng.set_profiling(True)
    eng.reset_kernel_times()
    for _ in range(ticks):
        eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
    eng.sync()
    kt = eng.kernel_times()
    eng.set_profiling(False)
    name, (launches, total_ms) = max(kt.items(), key=lambda kv: kv[1][1])
    avg_s = total_ms / launches / 1e3
    units = kernel_units(snap)
    leases_k, res_k = units[name]
    alg = algorithmic_bytes(leases_k, res_k, kernel_lease_bytes(name, leases_k, dense_frac))
    return {"kernel": name, "ticks": ticks, "warm_ticks": n, "avg_launch_us": round(avg_s * 1e6, 2),
            "achieved": round(alg / avg_s / 1e9, 1), "frac": round(alg / avg_s / 1e9 / HBM_PEAK_GBS, 4),
            "note": "the same kernel and store after the timed rounds, ticked back to back with no PCIe update "
                    "between; the step's roofline above is the kernel as the streaming step runs it, between "
                    "the rounds' store updates"}


def workload_line(name, snap, run, steps, single_kernel_tick):
    """One workload's numbers for the bench line's `extra` (or the line itself): rate,
    step time, the tick's fraction of HBM spec over its algorithmic bytes, per-class
    event times, the dominant kernel's roofline."""
    N = len(snap["wants"])
    t_step = run["elapsed"] / steps
    return {"workload": WORKLOADS[name], "value": N / t_step, "unit": "leases/s", "steps": steps,
            "ms_per_step": t_step * 1e3,
            **tick_fracs(snap, run["dense_frac"], t_step),
            "host_enqueue_us_per_step": round(run["host_enqueue_s"] / steps * 1e6, 2),
            "kernels": {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)}
                        for k, v in run["ktimes"].items()},
            "roofline": roofline_of(name, snap, run, steps, single_kernel_tick)}


def dist_fields(dist_info, run):
    """The N > 1 line's `dist`: torch's process group, what the library's own RCCL
    communicator reports on every rank (null in a gloo rehearsal), per-rank step times,
    the gather's time on the exchange stream, and the exchange's self-check."""
    ranks = run["ranks"]
    steps = [r["step_us"] for r in ranks]
    ex = [r["exchange_us"] for r in ranks if r["exchange_us"] is not None]
    d = dict(dist_info or {})
    d.update({"rccl_nranks": [r["rccl_nranks"] for r in ranks], "rccl_rank": [r["rccl_rank"] for r in ranks],
              "step_us_min": round(min(steps), 2), "step_us_max": round(max(steps), 2),
              "exchange_us": round(max(ex), 2) if ex else None,
              "exchange_us_note": "HIP events around the gather of the servers' blocks (ncclAllGather) on the "
                                  "exchange stream, profiled steps, max over ranks"})
    if run.get("self_check"):
        d.update({"consistent": run["self_check"]["consistent"], "check_sample": run["self_check"]["sample"],
                  "exchange_check": run["self_check"]})
    return d


def c2_shard_step(torch, Engine, dev_index, args, world, rank, sync_ranks, steps):
    """One rank's range of configs[2] (c2_bounds): back-to-back writeback ticks timed as
    every bench step (timed_steps); returns the rank's numbers."""
    from doorman_amd import workloads as W
    from doorman_amd.hierarchy import tick_cost
    snap = make_workload("c2", rank, world, "sharded", args.c2_partition)
    eng = Engine(dev_index, args.lib)
    try:
        eng.load(snap)
        now = W.NOW_NS
        step = lambda: eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
        run = timed_steps(torch, eng, step, steps, args.warmup, sync_ranks)
        sizes = np.diff(snap["seg_off"])
        return {"rank": rank, "resources": len(sizes), "leases": int(sizes.sum()),
                "predicted_bytes": int(tick_cost(sizes).sum()),
                "step_us": round(run["elapsed"] / steps * 1e6, 2),
                "kernels": {k: round(v[1] / max(v[0], 1) * 1e3, 2) for k, v in run["ktimes"].items()},
                "elapsed_s": run["elapsed"]}
    finally:
        eng.close()


def shard_summary(world, per_rank, steps, partition):
    """Whole-node numbers of a sharded configs[2] run from every rank's own numbers."""
    t = [r["step_us"] for r in per_rank]
    pb = [r["predicted_bytes"] for r in per_rank]
    n = sum(r["leases"] for r in per_rank)
    out = {"node_gpus": world, "leases_total": n,
           "step_us_max": max(t), "step_us_min": min(t), "step_max_over_min": round(max(t) / min(t), 4),
           "predicted_bytes_max_over_mean": round(max(pb) / (sum(pb) / len(pb)), 4),
           "partition": partition,
           "partition_note": {"classes": "hierarchy.assign_by_class: within every size class longest-processing-"
                                         "time-first over hierarchy.tick_cost (28 B per lease + 97 B per resource), "
                                         "then the smallest resources move until every rank holds the mean bytes",
                              "lpt": "hierarchy.assign_lpt: longest-processing-time-first over all resources",
                              "contiguous": "contiguous resource-id ranges balanced by hierarchy.tick_time"}[partition],
           "ranks": per_rank}
    if partition == "contiguous":
        out["bounds"] = [int(x) for x in c2_bounds(world)]
    return out


def rehearse_c2_shards(torch, Engine, dev_index, args, world, ranks):
    """--workload c2 --rehearse-shard N: the listed ranks' shards of an N-GPU configs[2]
    node, one after another on this GPU (each alone on the GPU, as on its own GPU of the
    node; no collective: the shards are independent)."""
    per = [c2_shard_step(torch, Engine, dev_index, args, world, k, lambda w, v: v, args.steps) for k in ranks]
    out = {"metric": "rehearsal: every rank's step of an N-GPU configs[2] node, one after another on one GPU "
                     "(not a bench line)", "steps": args.steps, "warmup": args.warmup,
           "workload": WORKLOADS["c2"] + f"; one snapshot sharded by resource id over {world} GPUs"}
    out.update(shard_summary(world, per, args.steps, args.c2_partition) if len(per) == world else {"ranks": per})
    if len(per) == world:
        out["projected_node_leases_per_s"] = out["leases_total"] / (out["step_us_max"] * 1e-6)
    return out


def c2_sharded_line(torch, Engine, dev_index, args, world, rank, sync_ranks, dist, red_dev):
    """N > 1: configs[2] over the node, every rank its range (strong scaling, no
    collective on the data path); value = all ranks' leases / the max over ranks of the
    timed region (barrier + synchronize on both sides, as the main line)."""
    mine = c2_shard_step(torch, Engine, dev_index, args, world, rank, sync_ranks, args.steps)
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    t = max(r["elapsed_s"] for r in allr)
    out = {"workload": WORKLOADS["c2"] + f"; one snapshot sharded by resource id over {world} GPUs",
           "value": sum(r["leases"] for r in allr) * args.steps / t, "unit": "leases/s",
           "ms_per_step": t / args.steps * 1e3, "scaling": "strong"}
    out.update(shard_summary(world, allr, args.steps, args.c2_partition))
    return out


def spawn_ranks(args) -> int:
    """--gpus N > 1 outside torchrun: start N ranks with torch.distributed.run before
    this process touches the GPU (a child process, never exec), return their status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=DEFAULT_WORKLOAD, choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the extra C1 line of the default run")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) on a node; gloo + --same-device rehearses N>1 on one GPU")
    ap.add_argument("--same-device", action="store_true", help="every rank on cuda:0 (rehearsal only)")
    ap.add_argument("--hier", default="auto", choices=["auto", "on", "off"],
                    help="every step also runs the intermediate-server exchange (SURVEY.md §8e, configs[3]): "
                         "publish totals, RCCL all-gather, root apportionment, take grants; auto = on for c3")
    ap.add_argument("--layout", default="auto", choices=["auto", "sharded", "replicated"],
                    help="c3 over N GPUs: sharded = one 100M-lease snapshot split by resource id (configs[3], "
                         "strong scaling; auto); replicated = a full store per GPU (weak scaling)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run each step's exchange before its leaf tick on one stream instead of beside the next tick")
    ap.add_argument("--rehearse-shard", type=int, default=0, metavar="N",
                    help="c3 only, one process on one GPU: run rank --rehearse-rank's full step of an N-GPU node "
                         "(its shard of the 100M-lease snapshot, the leaf tick with its publish, an N-block gathered "
                         "buffer -- the other N-1 blocks synthesized from their shards' totals, this rank's block "
                         "copied in place of the RCCL all-gather -- and the root round), on the exchange's own stream "
                         "as at N > 1; prints the rank's step time (not a whole-node measurement)")
    ap.add_argument("--rehearse-rank", type=int, default=0)
    ap.add_argument("--c2-partition", default="classes", choices=C2_PARTITIONS,
                    help="configs[2] over N GPUs: classes (every rank 1/N of every size class, bytes balanced), lpt "
                         "(longest-processing-time-first over all resources) or contiguous resource-id ranges "
                         "(weighted by the classes' measured rates)")
    ap.add_argument("--exchange", default="native", choices=["native", "python"],
                    help="native: each step is one library call (dm_hier_step: the leaf tick, then the block "
                         "gathered by the library's own RCCL communicator and the root round on the exchange "
                         "stream); python: the same sequence from Python (torch.distributed all-gather)")
    ap.add_argument("--no-busy-probe", action="store_true",
                    help="configs[4]: skip roofline.busy_gpu (tools/gpu_profile.sh: the profile then holds the "
                         "streaming step's ticks only)")
    ap.add_argument("--c4-sync-apply", action="store_true",
                    help="configs[4]: each round's batch through the synchronous dm_store_apply (A/B against the "
                         "default dm_store_apply_async)")
    ap.add_argument("--lib", default=None,
                    help="A/B only: another build of the same ABI (tools/ab_libs/*.so) for every engine of the run")
    ap.add_argument("--check-corrupt", action="store_true",
                    help="test only: the exchange self-check's step corrupts one rank's gathered copy (expect "
                         "dist.consistent false)")
    args = ap.parse_args()
    if args.rehearse_shard:
        if args.workload not in ("c2", "c3") or args.gpus != 1 or args.rehearse_shard < 2:
            raise SystemExit("--rehearse-shard N (N >= 2) rehearses ranks of an N-GPU configs[3] (c3) or configs[2] "
                             "(c2) node on one GPU: --workload c3|c2, --gpus 1")
        if args.workload == "c2":
            if not -1 <= args.rehearse_rank < args.rehearse_shard:
                raise SystemExit("--rehearse-rank must be in [0, N), or -1 for every rank in turn")
            args.layout, args.hier = "sharded", "off"
        else:
            if not 0 <= args.rehearse_rank < args.rehearse_shard:
                raise SystemExit("--rehearse-rank must be in [0, N)")
            args.layout, args.hier = "sharded", "on"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    hier = args.hier == "on" or (args.hier == "auto" and args.workload == "c3")
    layout = args.layout if args.layout != "auto" else ("sharded" if args.workload in ("c2", "c3") else "replicated")
    if layout == "sharded" and args.workload not in ("c2", "c3"):
        raise SystemExit("--layout sharded splits one snapshot by resource id: configs[3] (c3) or configs[2] (c2)")
    if layout == "sharded" and args.workload == "c2" and hier:
        raise SystemExit("configs[2] has no hierarchy: --hier off")

    import torch  # loaded first: libdoorman_hip then binds to torch's HIP runtime
    import torch.distributed as dist

    dev_index = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_index)
    gloo = args.dist_backend == "gloo"
    dist_info = None
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "device": "cuda:0 for every rank (rehearsal)" if args.same_device else "cuda:LOCAL_RANK"}
    red_dev = "cpu" if gloo else "cuda"

    def sync_ranks(what, v):
        if world <= 1:
            return v
        if what == "barrier":
            dist.barrier()
            return v
        t = torch.tensor([v], dtype=torch.int64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    from doorman_amd import workloads as W
    from doorman_amd.engine import Engine

    def gather(src, dst):
        if world > 1 and not gloo:
            dist.all_gather_into_tensor(dst, src)  # RCCL over xGMI
        elif world > 1:  # rehearsal: through host memory
            parts = [torch.empty_like(src, device="cpu") for _ in range(world)]
            dist.all_gather(parts, src.cpu())
            dst.copy_(torch.cat(parts).to(dst.device))
        else:
            dst.copy_(src)

    # the node this rank's shard belongs to: the real one, or the rehearsed one
    s_world, s_rank = (args.rehearse_shard, args.rehearse_rank) if args.rehearse_shard else (world, rank)

    def rehearsal_gather(stride):
        """--rehearse-shard: the gathered buffer of an s_world-rank node as this rank sees
        it.  The other ranks' blocks are synthesized once from their shards' initial
        totals ({SumWants, Count} per resource, no flags); each step copies this rank's
        block into its slot, where the RCCL all-gather would put it (the transfer itself
        is not rehearsed)."""
        b = c3_bounds(s_world)
        blocks = np.zeros((s_world * stride, 2))
        for j in range(s_world):
            if j == s_rank:
                continue
            sj = W.uniform_range(C3_R, C3_CLIENTS, int(b[j]), int(b[j + 1]), kind=W.FAIR_SHARE, seed=3)
            n = int(b[j + 1] - b[j])
            blocks[j * stride + 1: j * stride + 1 + n, 0] = sj["agg_sum_wants"]
            blocks[j * stride + 1: j * stride + 1 + n, 1] = np.asarray(sj["agg_count"], np.int64).view(np.float64)
        state = {"filled": False}

        def gather(src, dst):
            if not state["filled"]:
                dst.copy_(torch.from_numpy(blocks).to(dst.device))
                state["filled"] = True
            dst[s_rank * stride:(s_rank + 1) * stride].copy_(src)
        return gather

    exchange_used = {"mode": None}

    def exchange_mode(stride):
        """How the exchange runs: (native mode, RCCL id) for HierarchicalTick."""
        if args.exchange == "python" or args.no_pipeline:
            exchange_used["mode"] = "python"
            return None, None
        if world > 1 and gloo:  # the rehearsal of N ranks on one GPU: through host memory, from Python
            exchange_used["mode"] = "python (gloo)"
            return None, None
        if world > 1:  # one RCCL communicator of the library's own, its id from rank 0
            from doorman_amd.hierarchy import rccl_unique_id
            # every rank first checks that the library can load RCCL (dlopen, an id), and the
            # ranks agree before any of them enters the collective communicator set-up: a
            # rank that failed inside it would leave the others waiting there
            try:
                uid, ok = rccl_unique_id(), 1
            except Exception as e:  # noqa: BLE001 (reported, then the agreed fallback)
                print(f"[bench] rank {rank}: the library's RCCL is unavailable ({e})", file=sys.stderr, flush=True)
                uid, ok = None, 0
            if -sync_ranks("max_int", -ok) == 0:
                exchange_used["mode"] = "python (torch.distributed all-gather: the library's RCCL is unavailable)"
                return None, None
            obj = [uid if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            exchange_used["mode"] = "native (dm_hier_step, library RCCL all-gather over xGMI)"
            return "rccl", obj[0]
        exchange_used["mode"] = "native (dm_hier_step" + (", rehearsal: local copy of this rank's block)"
                                                          if args.rehearse_shard else ")")
        return "local", None

    def measure(layout):
        """Load this rank's store (and root copy), run the timed steps; returns the run,
        the snapshot and the engines (closed by the caller)."""
        snap = make_workload(args.workload, s_rank, s_world, layout, args.c2_partition)
        R = len(snap["seg_off"]) - 1
        eng = Engine(dev_index, args.lib)
        eng.load(snap)
        now = W.NOW_NS
        # back-to-back ticks: a forked tick's class streams join lazily (DM_DEFER_JOIN)
        step = lambda: eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
        root = ht = None
        if args.workload == "c4":
            step = streaming_step(eng, snap, rank, 2 * args.steps + args.warmup + 1, not args.c4_sync_apply)
        if hier:
            from doorman_amd.hierarchy import HierarchicalTick, root_snapshot
            root = Engine(dev_index, args.lib)
            if layout == "sharded":  # the root of the whole snapshot: one row per resource (its owner's)
                bounds = c3_bounds(s_world)
                root.load(root_snapshot(C3_R, 1, W.FAIR_SHARE, 1000.0, lease_length_s=20))
                stride = 1 + int(np.diff(bounds).max())
                native, comm_id = exchange_mode(stride)
                gfn = rehearsal_gather(stride) if args.rehearse_shard else gather
                # an exchange on a stream of its own gets a whole tick to finish before the leaf
                # takes its templates (two ticks of lag: HierarchicalTick's default then)
                ht = HierarchicalTick(torch, eng, root, C3_R, s_world, s_rank, gfn, shard_lo=bounds,
                                      pipelined=not args.no_pipeline, native=native, comm_id=comm_id)
                if native == "local" and args.rehearse_shard:  # the other ranks' blocks, synthesized once
                    gfn(ht.totals[0], ht.gathered[0])
            else:
                root.load(root_snapshot(R, world, W.FAIR_SHARE, np.asarray(snap["capacity"]) * world,
                                        lease_length_s=20))
                ht = HierarchicalTick(torch, eng, root, R, world, rank, gather, pipelined=not args.no_pipeline)
            step = lambda: ht.tick(now, asynchronous=True)  # noqa: E731
        run = timed_steps(torch, eng, step, args.steps, args.warmup, sync_ranks, extra_warm=args.workload != "c4",
                          also=[root] if root is not None else [])
        run["dense_frac"] = tick_dense_fraction(eng, snap, step)
        run["last_now"] = getattr(step, "last_now", now)
        if hasattr(step, "finish"):
            step.finish()  # the C4 rounds' asynchronous batches: retired, none rejected
        run["parts"] = int(eng.plan_info().get("stream_parts", 1))
        if ht is not None:
            ht.sync()
            ht.check()  # any server whose request the root rejected (server.go:863-866) fails loudly
            if layout == "sharded":
                run["self_check"] = exchange_self_check(torch, dist, ht, eng, root, c3_bounds(s_world), rank, world,
                                                        s_rank, now, red_dev, corrupt=args.check_corrupt)
        # what every rank saw: its step time, the ranks its RCCL communicator counts (the
        # library's own, not torch's process group), the gather's HIP-event time on the
        # exchange stream (profiled steps)
        g = run["ktimes"].get("hier_gather")
        comm = ht.comm_info() if ht is not None else None
        mine = {"rank": rank, "step_us": run["elapsed"] / args.steps * 1e6,
                "rccl_nranks": comm[0] if comm else None, "rccl_rank": comm[1] if comm else None,
                "exchange_us": g[1] / g[0] * 1e3 if g and g[0] else None}
        if world > 1:
            allr = [None] * world
            dist.all_gather_object(allr, mine)
        else:
            allr = [mine]
        run["ranks"] = allr
        t = torch.tensor([run["elapsed"]], dtype=torch.float64, device=red_dev)
        n = torch.tensor([len(snap["wants"])], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(n, op=dist.ReduceOp.SUM)
        run["t_max"], run["n_total"] = float(t.item()), float(n.item())
        return run, snap, eng, root

    if args.rehearse_shard and args.workload == "c2":
        ranks = range(s_world) if args.rehearse_rank < 0 else [s_rank]
        print(json.dumps(rehearse_c2_shards(torch, Engine, dev_index, args, s_world, ranks)), flush=True)
        return

    run, snap, eng, root = measure(layout)
    R, N = len(snap["seg_off"]) - 1, len(snap["wants"])
    t_max, n_total = run["t_max"], run["n_total"]
    roofline = roofline_of(args.workload, snap, run, args.steps,
                           single_kernel_tick=not hier and args.workload != "c4")
    if args.workload == "c4" and roofline is not None and not args.no_busy_probe:
        roofline["busy_gpu"] = busy_kernel_probe(eng, snap, run["last_now"], run["dense_frac"])
    now = W.NOW_NS

    extra = {}
    if args.rehearse_shard:
        args.no_extra = True
        args.no_cpu_baseline = True
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(snap, now, args.cpu_budget)
    if rank == 0 and world == 1 and not args.no_extra and args.workload == "c3":
        # the other single-GPU configurations beside the north-star line: configs[1] (C1),
        # configs[2] (C2, the Zipf load-imbalance stress) and configs[4]'s per-GPU streaming
        # store (C4: 10 rounds by default, each round's update batch held in pinned memory)
        eng.close()
        if root is not None:
            root.close()
            root = None
        for name in ("c1", "c2", "c4"):
            snapx = make_workload(name, 0)
            ex = Engine(dev_index, args.lib)
            ex.load(snapx)
            if name == "c4":
                kx = min(args.steps, 10)
                stx = streaming_step(ex, snapx, 0, 2 * kx + args.warmup + 1)
            else:
                kx = args.steps
                stx = lambda: ex.apportion(now, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
            rx = timed_steps(torch, ex, stx, kx, args.warmup, sync_ranks, extra_warm=name != "c4")
            rx["dense_frac"] = tick_dense_fraction(ex, snapx, stx)
            if hasattr(stx, "finish"):
                stx.finish()
            rx["parts"] = int(ex.plan_info().get("stream_parts", 1))
            extra[name] = workload_line(name, snapx, rx, kx, single_kernel_tick=name == "c1")
            if name == "c4" and extra[name]["roofline"] is not None:
                extra[name]["roofline"]["busy_gpu"] = busy_kernel_probe(ex, snapx, stx.last_now, rx["dense_frac"])
            extra[name]["aux_own_queues"] = bool(ex.plan_info().get("aux_own_queues", 0))
            ex.close()
            del snapx

    eng.close()
    if root is not None:
        root.close()
    if world > 1 and layout == "sharded" and not args.no_extra:
        # weak scaling beside the configs[3] line: every GPU its own full 100M-lease store
        rw, snapw, ew, rootw = measure("replicated")
        extra["weak_scaling"] = {"layout": "replicated: a full 100k x 1k store per GPU, every GPU an intermediate "
                                           "server of the same resources",
                                 "value": rw["n_total"] * args.steps / rw["t_max"], "unit": "leases/s",
                                 "leases_per_gpu": len(snapw["wants"]), "ms_per_step": rw["t_max"] / args.steps * 1e3,
                                 "scaling": "weak"}
        ew.close()
        if rootw is not None:
            rootw.close()

    if world > 1 and args.workload == "c3" and not args.no_extra:
        # configs[2]'s Zipf population over the node: every rank its cost-balanced range of
        # the one 1M-resource snapshot, no data-path collective (strong scaling)
        extra["c2_sharded"] = c2_sharded_line(torch, Engine, dev_index, args, world, rank, sync_ranks, dist, red_dev)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": n_total * args.steps / t_max,
            "unit": "leases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": run["warm_run"],
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if layout == "sharded" else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded numpy generators of SURVEY.md §8d)",
            "config": {"workload": WORKLOADS[args.workload] + (
                           (f"; one snapshot sharded by resource id over {world} GPU(s) (contiguous ranges), each GPU "
                            f"the intermediate server of its range" if layout == "sharded" else
                            "; every GPU holds a full store and is an intermediate server of the same resources")
                           + (f"; every step the exchange: publish per-resource totals, all-gather "
                              f"{'(RCCL) ' if world > 1 and not gloo else ''}of {world} block(s), the root's round "
                              + ("over this GPU's own resource range (only its owner requests a resource)"
                                 if layout == "sharded" else "over every resource on each GPU")
                              + ", this server's grants"
                              + ("" if args.no_pipeline else ", pipelined beside the next leaf tick (one tick of "
                                                             "lag, dm_hier_pipeline)") if hier else "")),
                       "layout": layout, "resources_per_gpu": R, "leases_per_gpu": N, "leases_total": int(n_total),
                       "parallelism": (f"intermediate-server hierarchy x{world}, {layout}" if hier
                                       else f"resource-sharded x{world} (no data-path collective)"),
                       "writeback": True},
            "exchange": exchange_used["mode"] if hier else None,
            # (a rehearsal reports its exchange self-check too: one rank of the rehearsed node)
            "dist": dist_fields(dist_info, run) if world > 1 or args.rehearse_shard else None,
            **tick_fracs(snap, run["dense_frac"], t_max / args.steps),
            "host_enqueue_us_per_step": round(run["host_enqueue_s"] / args.steps * 1e6, 2),
            "kernels": {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)}
                        for k, v in run["ktimes"].items()},
            "roofline": roofline,
            "extra": extra or None,
            "cpu_baseline": cpu,
        }
        if args.rehearse_shard:
            line["metric"] = "rehearsal: one rank's step of an N-GPU configs[3] node on one GPU (not a bench line)"
            line["value"] = N * args.steps / t_max
            line["unit"] = "leases/s of this rank"
            line["rehearsal"] = {
                "node_gpus": s_world, "rank": s_rank, "shard_resources": R, "shard_leases": N,
                "step_us": round(t_max / args.steps * 1e6, 2),
                "gather": "this rank's block copied into its slot of an N-block buffer (the other N-1 synthesized "
                          "once from their shards' totals); the RCCL transfer itself is not rehearsed",
                "projected_node_leases_per_s_if_ranks_alike": s_world * N * args.steps / t_max}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
