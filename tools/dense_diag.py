"""Dense-state diagnostic: which form each workgroup bin ran, tick by tick.

  python tools/dense_diag.py [--workload c2] [--ticks 5]

Loads the workload, runs writeback ticks at one instant (as bench.py does) with
per-class timing on, and prints after each tick the dense resources (dm_store_stats)
against the workgroup-bin resources, and the per-class launches and milliseconds.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (one HIP runtime)

from bench import make_workload  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--ticks", type=int, default=5)
    a = ap.parse_args()
    snap = make_workload(a.workload, 0)
    sizes = np.diff(np.asarray(snap["seg_off"]))
    group = int(((sizes >= 257) & (sizes <= 4096)).sum())
    eng = Engine(0)
    eng.load(snap)
    print(f"{a.workload}: {len(sizes)} resources, {group} in the workgroup bins; plan {eng.plan_info()}")
    eng.set_profiling(True)
    for t in range(a.ticks):
        eng.reset_kernel_times()
        eng.apportion(W.NOW_NS, writeback=True)
        eng.sync()
        kt = eng.kernel_times()
        print(f"tick {t}: {eng.store_stats()}")
        print("   " + "  ".join(f"{k} {v[0]}x{1000 * v[1]:.1f}us" for k, v in sorted(kt.items())))
    eng.close()


if __name__ == "__main__":
    main()
