"""Benchmark: client leases apportioned per second (whole node) + % of HBM peak.

One step = one apportionment tick over every lease of the rank's store: the
device-resident snapshot is decided (Clean, learning mode, the resource's
algorithm) and written back (DM_WRITEBACK), inputs already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c1ps|c2|c3]

For N > 1 it runs under torch.distributed.run, one rank per GPU; resources are
sharded by id (each rank owns its own shard of the workload: weak scaling, no
data-path collective).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_COPY_CEIL_GBS = 6290.0  # measured float4 copy ceiling (same table)
METRIC = "client leases apportioned/sec (whole node) + % HBM peak, FairShare, 1-8 GPU"

WORKLOADS = {
    "c1": "C1 (BASELINE configs[1]): 10,000 resources x 1,000 clients per GPU (10M leases), FairShare, uniform wants",
    "c1ps": "C1 (BASELINE configs[1]): 10,000 resources x 1,000 clients per GPU (10M leases), ProportionalShare",
    "c2": "C2 (BASELINE configs[2]): 1M resources, Zipf 1..1M clients (13,970,034 leases), mixed kinds, 5% learning",
    "c3": "C3 shape on one GPU (north-star target): 100,000 resources x 1,000 clients (100M leases), FairShare",
    "c4": "C4 (BASELINE configs[4]) per GPU: 125M-lease device-resident store (1B over 8 GPUs), 125k resources x "
          "1k client slots, FS/PS mixed, 5% learning; every step = 5 s refresh tick: 10% wants updates and 1% "
          "departures + 1% new clients over PCIe, then the tick",
}


def make_workload(name: str, rank: int):
    from doorman_amd import workloads as W
    if name == "c1":
        return W.c1(seed=1 + 1000 * rank, kind=W.FAIR_SHARE)
    if name == "c1ps":
        return W.c1(seed=1 + 1000 * rank, kind=W.PROPORTIONAL_SHARE)
    if name == "c2":
        return W.c2(seed=2 + 1000 * rank)
    if name == "c3":
        return W.uniform(100_000, 1_000, kind=W.FAIR_SHARE, seed=3 + 1000 * rank)
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


LEASE_BYTES = 44  # read wants 8 + has 8 + subclients 4 + expiry 8, write gets 8 + expiry 8


def algorithmic_bytes(n_leases: int, n_resources: int) -> int:
    # BASELINE.md §3 / SURVEY.md §8(d) per lease: read wants, has, subclients, expiry; write
    # gets, expiry.  The device table holds subclients as int32 (the boundary already
    # restricts them to [0, 2^31)), so a lease is 44 B, not the 48 B of an int64 column;
    # per resource config + offsets + outputs (64 B).  Re-reads are not counted.
    return LEASE_BYTES * n_leases + 64 * n_resources


def kernel_units(eng, snap):
    """(leases, resources) each kernel class of the plan processes per launch."""
    so = snap["seg_off"]
    sizes = np.diff(so)
    units = {}
    edges = [("group16", 9, 16), ("group32", 17, 32), ("wave64x1", 33, 64), ("wave64x2", 65, 128),
             ("wave64x4", 129, 256), ("block256x2", 257, 512), ("block256x4", 513, 1024), ("block512x4", 1025, 2048),
             ("block1024x4", 2049, 4096)]
    small = sizes <= 8
    units["small_packed"] = (int(sizes[small].sum()), int(small.sum()))
    for name, lo, hi in edges:
        m = (sizes >= lo) & (sizes <= hi)
        units[name] = (int(sizes[m].sum()), int(m.sum()))
    big = sizes > 4096
    for name in ("large_a", "large_b", "large_c", "large_map", "large_fin", "general"):
        units[name] = (int(sizes[big].sum()), int(big.sum()))
    return units


def streaming_step(eng, snap, rank, n_ticks):
    """configs[4]: one 5 s refresh tick of a device-resident store.  Per tick the
    host sends 10% wants updates (row mask + packed values, narrow Assign), releases
    1% of the clients (departures, store.go:142-151), inserts 1% new clients into
    free slots (upsert onto released rows) -- all three in one dm_store_apply call --
    then the tick runs with writeback.  The update batches (what the RPCs would deliver) are generated
    before the timed region."""
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
        # per update at 10% instead of an 8-B row index: dm_store_update_wants_mask)
        cols = (W.rows_to_mask(upd, N), rng.uniform(0.5, 1.5, len(upd)), gone, new, np.zeros(k),
                rng.uniform(0.5, 1.5, k), np.ones(k, np.int64), np.full(k, now + 3600 * W.NS, np.int64))
        # the RPC layer would decode requests straight into page-locked buffers
        # (dm_host_alloc), which then cross PCIe by DMA
        pinned = []
        for a in cols:
            h = eng.host_empty(len(a), a.dtype)
            h[:] = a
            pinned.append(h)
        batches.append((*pinned, now))
    it = iter(batches)

    def step():
        mask, w, gone, new, nh, nw, ns, ne, t = next(it)
        eng.apply(mask, w, gone, (new, nh, nw, ns, ne))  # the round's three update kinds, one call
        eng.apportion(t, writeback=True, asynchronous=True)

    return step


def subset_rows(snap, max_rows):
    """the leading resources of a snapshot holding at most max_rows leases"""
    from doorman_amd import workloads as W
    so = snap["seg_off"]
    k = int(np.searchsorted(so, max_rows, side="right")) - 1
    return W.subset(snap, np.arange(max(k, 1)))


def cpu_baseline(snap, now_ns, budget_s=12.0):
    """Reference algorithm restated in C (oracle, literal per-request Resource.Decide on a
    private copy of the store, single thread), timed on a bounded sample of this workload."""
    from oracle import oracle as O
    so = snap["seg_off"]
    sizes = np.diff(so)
    order = np.argsort(-sizes, kind="stable")
    # sample whole resources from the middle of the size distribution up to the budget
    rng = np.random.default_rng(0)
    cand = rng.permutation(np.flatnonzero(sizes > 0))
    gets = np.empty(len(snap["wants"]))
    done_rows, t_total, used = 0, 0.0, []
    for r in cand:
        n = int(sizes[r])
        lo, hi = int(so[r]), int(so[r + 1])
        if n > 4000:  # O(n^2) per resource: take a slice of clients of the big resources
            hi = lo + 4000
        t0 = time.perf_counter()
        done_rows += O.apportion_literal_rows(snap, int(r), lo, hi, now_ns, gets)
        t_total += time.perf_counter() - t0
        used.append(int(r))
        if t_total > budget_s:
            break
    del order
    # the closed form (same outputs) over all resources on the
    # host's cores, the optimised-CPU comparator, timed on the whole snapshot
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    O.apportion(subset_rows(snap, 2000), now_ns, "closed", threads=threads)  # warm the pool
    reps, t_mt = 0, 0.0
    while reps < 3 and t_mt < 5.0:
        t0 = time.perf_counter()
        O.apportion(snap, now_ns, "closed", threads=threads)
        t_mt += time.perf_counter() - t0
        reps += 1
    return {
        "value": done_rows / t_total if t_total > 0 else None,
        "unit": "leases/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{done_rows} leases of {len(used)} resources of the same workload, each decided by the literal "
                  f"C restatement of Resource.Decide (go/server/doorman/resource.go:100-113) on a private store copy "
                  f"(O(n) per request as in the reference), single thread, {t_total:.1f} s",
        "closed_form_mt": {
            "value": reps * len(snap["wants"]) / t_mt,
            "unit": "leases/s",
            "cores": threads,
            "sample": f"whole snapshot x{reps}: oracle/ closed form (SURVEY.md §8a), OpenMP over resources",
        },
        "host": host_info(),
    }


def host_info():
    """CPU model and core counts of the box the baseline ran on (SURVEY.md §8d asks
    for them next to the Go reference's GOMAXPROCS, which has no counterpart here)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cores": usable}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) on a node; gloo + --same-device rehearses N>1 on one GPU")
    ap.add_argument("--same-device", action="store_true", help="every rank on cuda:0 (rehearsal only)")
    ap.add_argument("--hier", action="store_true",
                    help="every step runs the intermediate-server exchange first (SURVEY.md §8e, configs[3]): "
                         "publish totals, RCCL all-gather, root apportionment, take grants, then the leaf tick")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch  # loaded first: libdoorman_hip then binds to torch's HIP runtime
    import torch.distributed as dist

    dev_index = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_index)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))

    from doorman_amd import workloads as W
    from doorman_amd.engine import Engine

    snap = make_workload(args.workload, rank)
    R, N = len(snap["seg_off"]) - 1, len(snap["wants"])
    eng = Engine(dev_index)
    eng.load(snap)
    now = W.NOW_NS

    def barrier():
        if world > 1:
            dist.barrier()

    # back-to-back ticks: a forked tick's class streams join lazily (DM_DEFER_JOIN)
    step = lambda: eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
    root = None
    if args.workload == "c4":
        step = streaming_step(eng, snap, rank, 2 * args.steps + args.warmup)
    if args.hier:
        from doorman_amd.hierarchy import HierarchicalTick, root_snapshot
        root = Engine(dev_index)
        root.load(root_snapshot(R, world, W.FAIR_SHARE, np.asarray(snap["capacity"]) * world, lease_length_s=20))

        def gather(src, dst):
            if world > 1 and not gloo:
                dist.all_gather_into_tensor(dst, src)  # RCCL over xGMI
            elif world > 1:  # rehearsal: through host memory
                parts = [torch.empty_like(src, device="cpu") for _ in range(world)]
                dist.all_gather(parts, src.cpu())
                dst.copy_(torch.cat(parts).to(dst.device))
            else:
                dst.copy_(src)

        ht = HierarchicalTick(torch, eng, root, R, world, rank, gather)
        step = lambda: ht.tick(now, asynchronous=True)  # noqa: E731

    # W warmup steps, then more untimed steps until ~0.3 s of ticks have run: the
    # first few milliseconds of back-to-back ticks run ~10% slow (clock ramp; C3
    # measured 843 us/tick after 3 warmup ticks, 765 after 30).  The extra count is
    # agreed over ranks (the hierarchy's steps hold a collective).  C4's update
    # batches are pre-generated per step, so it runs exactly W.
    t_w = time.perf_counter()
    for _ in range(max(args.warmup, 1)):
        step()
    eng.sync()
    per_step = (time.perf_counter() - t_w) / max(args.warmup, 1)
    extra = 0 if args.workload == "c4" else min(20000, int(0.3 / max(per_step, 1e-6)))
    if world > 1:
        ex = torch.tensor([extra], dtype=torch.int64, device="cpu" if gloo else "cuda")
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        extra = int(ex.item())
    for i in range(extra):
        step()
        if i % 8 == 7:
            eng.sync()
    warm_run = max(args.warmup, 1) + extra
    eng.sync()
    # timed region: only a start/stop HIP event pair on the engine's stream
    ext = torch.cuda.ExternalStream(eng.stream)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(ext)
    for _ in range(args.steps):
        step()
    eng.join()  # every class stream's work before the closing event
    ev1.record(ext)
    eng.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    stream_ms = ev0.elapsed_time(ev1)
    # profiled region (same steps): HIP events around every kernel launch, on the
    # stream each kernel runs on, for the per-kernel roofline
    eng.set_profiling(True)
    eng.reset_kernel_times()
    for _ in range(args.steps):
        step()
    eng.sync()
    ktimes = eng.kernel_times()
    eng.set_profiling(False)
    red_dev = "cpu" if gloo else "cuda"
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    n = torch.tensor([N], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
    t_max, n_total = float(t.item()), float(n.item())

    # dominant kernel: largest share of in-stream time
    units = kernel_units(eng, snap)
    dom = max(ktimes.items(), key=lambda kv: kv[1][1]) if ktimes else None
    roofline = None
    if dom:
        name, (launches, total_ms) = dom
        avg_s = total_ms / launches / 1e3
        single = len(ktimes) == 1 and launches == args.steps and not args.hier and args.workload != "c4"
        if single:  # one kernel per tick: HIP events around the timed region itself
            avg_s = stream_ms / args.steps / 1e3
        leases_k, res_k = units.get(name, (N, R))
        alg = algorithmic_bytes(leases_k, res_k)
        achieved = alg / avg_s / 1e9
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
        if os.path.exists(pmc_path):
            try:
                traffic = json.load(open(pmc_path)).get(name, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roofline = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "frac_of_copy_ceiling": round(achieved / HBM_COPY_CEIL_GBS, 4), "traffic": traffic,
                    "algorithmic_bytes_per_launch": alg, "avg_launch_us": round(avg_s * 1e6, 2),
                    "kernel_time_share": round(total_ms / sum(v[1] for v in ktimes.values()), 3),
                    "timed_region_stream_us_per_step": round(stream_ms * 1e3 / args.steps, 2),
                    "duration_source": ("HIP event pair around the timed region on the kernel's stream (one kernel "
                                        "per tick)" if single else "HIP events around every launch, profiled region")}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(snap, now, args.cpu_budget)

    if rank == 0:
        tick_bytes = algorithmic_bytes(N, R)
        line = {
            "metric": METRIC,
            "value": n_total * args.steps / t_max,
            "unit": "leases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm_run,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded numpy generators of SURVEY.md §8d)",
            "config": {"workload": WORKLOADS[args.workload] + (
                           "; hierarchical: every GPU is an intermediate server of the same resources, RCCL "
                           "all-gather of per-resource totals + root apportionment each step" if args.hier else ""),
                       "resources_per_gpu": R, "leases_per_gpu": N,
                       "parallelism": (f"intermediate-server hierarchy x{world} (all-gather 16 B x R per GPU)"
                                       if args.hier else f"resource-sharded x{world} (no data-path collective)"),
                       "writeback": True},
            "tick_hbm_frac": round(tick_bytes / (t_max / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
            "kernels": {k: {"launches": v[0], "avg_us": round(v[1] / max(v[0], 1) * 1e3, 2)} for k, v in ktimes.items()},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if root is not None:
        root.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
