"""Per-kernel times (HIP events around every launch) of one workload's tick,
for one or more library builds.

  python tools/kprof.py --workload c2 [--lib LIB.so ...] [--steps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

from bench import algorithmic_bytes, make_workload  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    snap = make_workload(args.workload, 0)
    for lib in args.lib or [None]:
        e = Engine(0, os.path.abspath(lib) if lib else None)
        e.load(snap)
        info = e.plan_info()
        for _ in range(3):
            e.apportion(W.NOW_NS, writeback=True)
        e.set_profiling(True)
        e.reset_kernel_times()
        for _ in range(args.steps):
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True)
        kt = e.kernel_times()
        e.close()
        print(os.path.basename(lib or "in-tree"), {k: v for k, v in info.items() if v})
        for k, (n, ms) in kt.items():
            print(f"   {k:14s} {ms / n * 1e3:9.1f} us")


if __name__ == "__main__":
    main()
