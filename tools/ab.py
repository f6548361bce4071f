"""Interleaved A/B timing of library builds in ONE process (cdna guide §5.4 rule 24).

  python tools/ab.py --workload c1 --rounds 8 --steps 20 LIB_A.so LIB_B.so[:inplace|:alternate][@VAR=value+...] ...

Every build gets its own context with the same snapshot; rounds alternate between
builds; per build the per-launch kernel time (HIP events) and the tick wall time
are reported as median and min over rounds.
"""
import argparse
import contextlib
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (one HIP runtime)

from bench import algorithmic_bytes, make_workload  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import c4_variants  # noqa: E402


@contextlib.contextmanager
def env(values):
    """Environment variables in force for one engine's calls (A/B knobs)."""
    saved = {k: os.environ.get(k) for k in values}
    os.environ.update(values)
    try:
        yield
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--workload", default="c1", help="a bench workload, or uRxC (R resources x C clients)")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--per-kernel", action="store_true", help="median us per tick of every kernel class")
    args = ap.parse_args()
    if args.workload.startswith("u") and "x" in args.workload:  # uRxC: R resources x C clients, FairShare
        nr, nc = (int(v) for v in args.workload[1:].split("x"))
        snap = W.uniform(nr, nc, kind=W.FAIR_SHARE, seed=3)
    elif args.workload in c4_variants.VARIANTS:  # a configs[4]-shaped store (tools/c4_variants.py)
        snap = c4_variants.make(**c4_variants.VARIANTS[args.workload])
    else:
        snap = make_workload(args.workload, 0)
    R, N = len(snap["seg_off"]) - 1, len(snap["wants"])
    engines = []
    for p in args.libs:
        spec, _, envs = p.partition("@")  # LIB[:mode][@VAR=value+...]: environment at the engine's creation
        path, _, mode = spec.partition(":")
        # VAR=value pairs split on "+" (a value may hold commas, e.g. DM_CU_PART=96,64,64,32)
        e_env = dict(kv.partition("=")[::2] for kv in filter(None, envs.split("+")))
        with env(e_env):
            e = Engine(0, os.path.abspath(path))
        e.env = e_env  # also in force around its ticks (knobs read per launch)
        e.wb_columns = mode if mode in ("inplace", "alternate") else "auto"
        e.load(snap)
        with env(e.env):
            for _ in range(3):
                e.apportion(W.NOW_NS, writeback=True, wb_columns=e.wb_columns)
        engines.append(e)
    res = {p: {"tick_us": [], "kern_us": [], "plain_us": [], "cls": {}} for p in args.libs}
    def one_round(p, e):
        e.set_profiling(True)
        e.reset_kernel_times()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True, wb_columns=e.wb_columns)
        e.sync()
        dt = time.perf_counter() - t0
        kt = e.kernel_times()
        e.set_profiling(False)
        res[p]["tick_us"].append(dt / args.steps * 1e6)
        torch.cuda.synchronize()  # the same ticks without per-kernel events
        t0 = time.perf_counter()
        for _ in range(args.steps):
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True, wb_columns=e.wb_columns)
        e.sync()
        res[p]["plain_us"].append((time.perf_counter() - t0) / args.steps * 1e6)
        res[p]["kern_us"].append(sum(v[1] for v in kt.values()) / args.steps * 1e3)
        for name, v in kt.items():
            res[p]["cls"].setdefault(name, []).append(v[1] / args.steps * 1e3)

    for _ in range(args.rounds):
        for p, e in zip(args.libs, engines):
            with env(e.env):
                one_round(p, e)
    alg = algorithmic_bytes(N, R)
    for p in args.libs:
        k = res[p]["kern_us"]
        t = res[p]["tick_us"]
        print(f"{os.path.basename(p):34s} kernel med {statistics.median(k):8.2f} us min {min(k):8.2f} "
              f"({alg / min(k) / 1e3:7.1f} GB/s best) | tick med {statistics.median(t):8.2f} us | "
              f"unprofiled tick med {statistics.median(res[p]['plain_us']):8.2f} min {min(res[p]['plain_us']):8.2f} us")
        if args.per_kernel:
            print("    " + "  ".join(f"{n} {statistics.median(v):.1f}" for n, v in sorted(res[p]["cls"].items())))
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
