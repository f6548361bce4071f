"""Diagnose a configs[2] shard against the oracle tick by tick (one process, one GPU).
usage: python tools/c2_shard_diag.py WORLD RANK TICKS [sync]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401

import bench  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402
from test_c2_full_gpu import _check, _host_tick, _pick  # noqa: E402

world, rank, ticks = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
sync_each = len(sys.argv) > 4
snap = bench.make_workload("c2", rank, world, "sharded")
so = np.asarray(snap["seg_off"])
pick = _pick(snap, np.random.default_rng(70 + rank))
host = W.subset(snap, pick)
eng = Engine(0)
eng.load(snap)
for t in range(ticks):
    eng.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
    _host_tick(host, W.NOW_NS)
    if sync_each or t == ticks - 1:
        eng.sync()
        try:
            _check(eng, host, pick, so, f"tick {t + 1}")
            print(f"tick {t + 1}: ok")
        except AssertionError as e:
            print(f"tick {t + 1}: {e}")
eng.close()
