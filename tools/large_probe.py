"""Large-resource class alone: per-kernel times of C2's resources > 4096 rows
(or the whole C2 tick with --all) for library builds and large-path modes.

  python tools/large_probe.py [--all] [--redo] LIB.so[:chain] ...

--redo: before every tick a wants refresh of each resource's first row (values
alternate), so every speculated resource fails its check and takes the redo.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--small", action="store_true", help="only the resources of <= 4096 rows")
    ap.add_argument("--sizes", default=None, help="LO-HI: only resources with LO <= rows <= HI")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--redo", action="store_true", help="every tick redoes every large resource")
    args = ap.parse_args()
    snap = W.c2()
    if not args.all:
        import numpy as np
        sizes = np.diff(snap["seg_off"])
        if args.sizes:
            lo, hi = (int(x) for x in args.sizes.split("-"))
            keep = (sizes >= lo) & (sizes <= hi)
        else:
            keep = (sizes <= 4096) if args.small else (sizes > 4096)
        snap = W.subset(snap, np.flatnonzero(keep))
    n = len(snap["wants"])
    import numpy as np
    first = np.asarray(snap["seg_off"])[:-1][np.diff(np.asarray(snap["seg_off"])) > 0]
    w_alt = [snap["wants"][first].copy(), snap["wants"][first] * 1.01 + 0.5]
    it = [0]

    def tick(e):
        if args.redo:
            it[0] += 1
            e.update_wants(first, w_alt[it[0] & 1])
        e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)

    for p in args.libs:
        p, _, envs = p.partition("@")  # LIB[:mode][@VAR=value,...]: environment for that engine
        for kv in filter(None, envs.split(",")):
            var, _, val = kv.partition("=")
            os.environ[var] = val
        path, _, mode = p.partition(":")
        e = Engine(0, os.path.abspath(path))
        e.load(snap)
        for _ in range(5):
            e.apportion(W.NOW_NS, writeback=True)
        e.set_profiling(True)
        e.reset_kernel_times()
        import time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tick(e)
        e.sync()
        dt = (time.perf_counter() - t0) / args.steps * 1e6
        kt = e.kernel_times()
        e.set_profiling(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tick(e)
        e.sync()
        dp = (time.perf_counter() - t0) / args.steps * 1e6
        e.close()
        for kv in filter(None, envs.split(",")):
            os.environ.pop(kv.partition("=")[0], None)
        ks = "  ".join(f"{k} {ms / cnt * 1e3:.1f}" for k, (cnt, ms) in sorted(kt.items()))
        print(f"{os.path.basename(p) + '@' + envs:40s} rows {n} tick {dt:7.1f} us, unprofiled {dp:7.1f} us | {ks}", flush=True)


if __name__ == "__main__":
    main()
