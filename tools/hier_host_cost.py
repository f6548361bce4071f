"""Probe: the host's cost of one dm_hier_step (native local exchange, G servers, sharded)
on a leaf small enough that the GPU finishes first -- the wall time per step is then
the host's enqueue path (ctypes, the library, HIP calls).
  python tools/hier_host_cost.py [G] [resources] [rows]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402
from doorman_amd.hierarchy import HierarchicalTick, partition, root_snapshot  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    R0 = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 600
    torch.cuda.set_device(0)
    sizes = np.full(R0 * G, rows)
    R = len(sizes)
    lo = partition(sizes, G)
    S = 1 + int(np.diff(lo).max())
    full = W.make_snapshot(sizes, 1.0, 0.0, 1, W.NOW_NS + 600 * W.NS, W.FAIR_SHARE, 1000.0)
    shard = W.subset(full, np.arange(lo[0], lo[1]))
    leaf, root = Engine(0), Engine(0)
    leaf.load(shard)
    root.load(root_snapshot(R, 1, W.FAIR_SHARE, 1000.0))
    ht = HierarchicalTick(torch, leaf, root, R, G, 0, None, shard_lo=lo, pipelined=True, native="local")
    for k in (200, 2000, 2000):
        t0 = time.perf_counter()
        c0 = time.thread_time()
        for _ in range(k):
            ht.tick(W.NOW_NS, asynchronous=True)
        t1 = time.perf_counter()
        c1 = time.thread_time()
        ht.sync()
        t2 = time.perf_counter()
        print(f"G={G} leaf {R0}x{rows}: {k} steps, enqueue {(t1 - t0) / k * 1e6:.2f} us/step wall "
              f"({(c1 - c0) / k * 1e6:.2f} CPU), total {(t2 - t0) / k * 1e6:.2f} us/step", flush=True)
    leaf.close()
    root.close()


if __name__ == "__main__":
    main()
