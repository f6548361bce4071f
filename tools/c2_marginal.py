"""configs[2]'s tick with one size class left out at a time: the marginal time of each
class in the shared tick (which class the tick waits for).
usage: python tools/c2_marginal.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

import bench  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402

full = bench.make_workload("c2", 0)
sizes = np.diff(full["seg_off"])
classes = {"tiles": (1, 4), "subs": (5, 256), "blocks": (257, 4096), "large": (4097, 1 << 62)}


def tick(snap, K=400):
    with Engine(0) as eng:
        eng.load(snap)
        step = lambda: eng.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
        for _ in range(600):
            step()
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        eng.sync()
        return round((time.perf_counter() - t0) / K * 1e6, 2)


out = {"all": tick(full)}
for name, (lo, hi) in classes.items():
    keep = np.flatnonzero(~((sizes >= lo) & (sizes <= hi)))
    out["without_" + name] = tick(W.subset(full, keep))
    only = np.flatnonzero((sizes >= lo) & (sizes <= hi))
    out["only_" + name] = tick(W.subset(full, only))
print(json.dumps(out), flush=True)
