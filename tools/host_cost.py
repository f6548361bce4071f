"""Host-side cost of enqueueing one asynchronous writeback tick (no GPU wait) vs
the tick's wall time, for a workload: is the tick bound by launches?

  python tools/host_cost.py --workload c2 [LIB.so]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import make_workload  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "doorman_amd", "libdoorman_hip.so"))
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    e = Engine(0, os.path.abspath(args.lib))
    e.load(make_workload(args.workload, 0))
    for _ in range(5):
        e.apportion(W.NOW_NS, writeback=True)
    torch.cuda.synchronize()
    enq = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
        enq.append(time.perf_counter() - a)
    e.sync()
    wall = (time.perf_counter() - t0) / args.steps
    enq.sort()
    print(f"{args.workload}: tick wall {wall * 1e6:.1f} us, host enqueue per tick median {enq[len(enq) // 2] * 1e6:.1f} "
          f"us (min {enq[0] * 1e6:.1f}, max {enq[-1] * 1e6:.1f}); plan {e.plan_info()}")
    e.close()


if __name__ == "__main__":
    main()
