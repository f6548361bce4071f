"""Probe: one rank's configs[3] shard (N-way) ticked alone, without the hierarchy's
exchange -- the leaf tick's own time at shard size, beside bench.py --rehearse-shard N.
  python tools/shard_leaf.py [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.cuda.set_device(0)
    snap = bench.make_workload("c3", 0, n, "sharded")
    with Engine(0, os.environ.get("DM_LIB") or None) as e:
        e.load(snap)
        st = lambda: e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
        for steps in (200, 200):
            r = bench.timed_steps(torch, e, st, steps, 20, lambda what, v: v)
            us = r["elapsed"] / steps * 1e6
            nb = len(snap["wants"]) * 24 + (len(snap["seg_off"]) - 1) * 97
            print(f"shard {n}: {len(snap['wants'])} leases, leaf tick alone {us:.2f} us "
                  f"({nb / us / 1e6:.2f} TB/s algorithmic)", flush=True)


if __name__ == "__main__":
    main()
