"""Host-side cost of a pipelined hierarchical step (C3 shape, one GPU).

  python tools/pipe_probe.py [--resources 100000] [--steps 200]

For the pipelined and unpipelined exchange: wall time per step over back-to-back
steps, and the host time spent inside each call of the step (the leaf tick's
enqueue, the exchange's enqueue).  A host call that takes about a tick's GPU time
blocks on the GPU, which leaves the GPU idle while the next launches are enqueued.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402
from doorman_amd.hierarchy import HierarchicalTick, root_snapshot  # noqa: E402


def run(R, steps, pipelined):
    snap = W.uniform_range(R, 1000, 0, R)
    leaf = Engine(0)
    leaf.load(snap)
    root = Engine(0)
    root.load(root_snapshot(R, 1, W.FAIR_SHARE, 1000.0, lease_length_s=20))
    ht = HierarchicalTick(torch, leaf, root, R, 1, 0, None, shard_lo=np.array([0, R]), pipelined=pipelined)
    for _ in range(30):
        ht.tick(W.NOW_NS, asynchronous=True)
    ht.sync()
    t_leaf, t_x = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        if pipelined:
            leaf.apportion(W.NOW_NS, writeback=True, asynchronous=True)
            b = time.perf_counter()
            ht.exchange(W.NOW_NS)
        else:
            ht.exchange(W.NOW_NS)
            b = time.perf_counter()
            leaf.apportion(W.NOW_NS, writeback=True, asynchronous=True)
        c = time.perf_counter()
        t_leaf.append((b - a) * 1e6 if pipelined else (c - b) * 1e6)
        t_x.append((c - b) * 1e6 if pipelined else (b - a) * 1e6)
    ht.sync()
    dt = (time.perf_counter() - t0) / steps * 1e6
    med = lambda v: float(np.median(v))  # noqa: E731
    print(f"R={R} pipelined={pipelined}: {dt:7.1f} us/step; host per call: leaf tick med {med(t_leaf):7.1f} "
          f"max {max(t_leaf):7.1f}, exchange med {med(t_x):7.1f} max {max(t_x):7.1f}", flush=True)
    leaf.close()
    root.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resources", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    for p in (True, False, True):
        run(args.resources, args.steps, p)


if __name__ == "__main__":
    main()
