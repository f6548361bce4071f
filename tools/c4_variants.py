"""configs[4]'s tick kernel without updates, one store property changed at a time: which
of C4's differences from configs[3] (mixed FS/PS kinds, 5 % learning, 2 % free slots,
125M rows) costs the dense kernel its rate.  Writeback ticks back to back (as
c4_probe's "fresh"), HIP-event kernel times.
usage: python tools/c4_variants.py [ticks] [variant ...]   (variant: a VARIANTS key or
bench_c3, optionally with _const: every tick at the same now; WARM=n warm-up ticks, default 4;
GAP_MS=x: the GPU idle x ms after each warm-up tick)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def make(free=0.02, learning=0.05, kind="mixed", R=125_000, wscale=1.0):
    snap = W.uniform(R, 1_000, kind=kind, seed=4)
    snap["wants"] *= wscale
    rng = np.random.default_rng(40)
    snap["learning_end_ns"] = np.where(rng.random(R) < learning, W.NOW_NS + 3600 * W.NS,
                                       W.INT64_MIN).astype(np.int64)
    f = rng.random(len(snap["wants"])) < free
    snap["wants"][f] = 0.0
    snap["has"][f] = 0.0
    snap["subclients"] = np.where(f, 0, 1).astype(np.int64)
    snap["expiry_ns"][f] = W.RELEASED
    snap["expiry_ns"][~f] = W.NOW_NS + 3600 * W.NS
    return W.add_store_sums(snap)


GAP_MS = 0.0
VARIANTS = {
    "c4": {},
    "no_free": {"free": 0.0},
    "no_learning": {"learning": 0.0},
    "fs_only": {"kind": W.FAIR_SHARE},
    "ps_only": {"kind": W.PROPORTIONAL_SHARE},
    "c3like": {"free": 0.0, "learning": 0.0, "kind": W.FAIR_SHARE},
    "c3like_ps": {"free": 0.0, "learning": 0.0, "kind": W.PROPORTIONAL_SHARE},
    "ps_free": {"learning": 0.0, "kind": W.PROPORTIONAL_SHARE},
    "fs_free": {"learning": 0.0, "kind": W.FAIR_SHARE},
    "ps_learn": {"free": 0.0, "kind": W.PROPORTIONAL_SHARE},
    "ps_free_over": {"learning": 0.0, "kind": W.PROPORTIONAL_SHARE, "wscale": 1.1},
    "ps_under": {"free": 0.0, "learning": 0.0, "kind": W.PROPORTIONAL_SHARE, "wscale": 0.9},
    "fs_under": {"free": 0.0, "learning": 0.0, "kind": W.FAIR_SHARE, "wscale": 0.9},
    "c1like_fs": {"free": 0.0, "learning": 0.0, "kind": W.FAIR_SHARE, "R": 10_000},
    "c1like_ps": {"free": 0.0, "learning": 0.0, "kind": W.PROPORTIONAL_SHARE, "R": 10_000},
    "c3like_100k": {"free": 0.0, "learning": 0.0, "kind": W.FAIR_SHARE, "R": 100_000},
}

def main():
    ticks = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    WARM = int(os.environ.get("WARM", "4"))  # noqa: N806
    global GAP_MS
    GAP_MS = float(os.environ.get("GAP_MS", "0"))
    names = sys.argv[2:] or list(VARIANTS)
    for name in names:
        const = name.endswith("_const")  # every tick at the same now (as tools/c2_marginal.py)
        base = name[:-6] if const else name
        if base == "bench_c3":
            import bench
            snap = bench.make_workload("c3", 0)
        else:
            snap = make(**VARIANTS[base])
        step = 0 if const else 5 * W.NS
        with Engine(0) as eng:
            eng.load(snap)
            t = W.NOW_NS
            for i in range(WARM):  # ~0.3 s of back-to-back ticks first (bench.timed_steps' extra warm-up)
                t += step
                eng.apportion(t, writeback=True, asynchronous=True, defer_join=True)
                if GAP_MS:  # (the GPU idle between warm-up ticks: tick count without sustained load)
                    eng.sync()
                    time.sleep(GAP_MS / 1e3)
                elif i % 8 == 7:
                    eng.sync()
            eng.sync()
            eng.set_profiling(True)
            eng.reset_kernel_times()
            t0 = time.perf_counter()
            for _ in range(ticks):
                t += step
                eng.apportion(t, writeback=True, asynchronous=True, defer_join=True)
            eng.sync()
            dt = (time.perf_counter() - t0) / ticks
            kt = {k: round(v[1] / max(v[0], 1) * 1e3, 2) for k, v in eng.kernel_times().items()}
            st = eng.store_stats()
        print(json.dumps({"variant": name, "tick_ms": round(dt * 1e3, 3), "kernels": kt,
                          "dense": st["dense_leases"], "rows": int(snap["seg_off"][-1])}), flush=True)
        del snap


if __name__ == "__main__":
    main()
