"""Tick time by resource size: uniform stores of n-row resources (mixed kinds as
configs[2]: 40% FS / 40% PS / 10% Static / 10% NoAlgorithm), back-to-back writeback
ticks as bench.py times them.  Prints one JSON line per size: us per tick, the byte
model's GB/s (28 B per lease + 97 B per resource) and the per-class event times.
usage: python tools/size_sweep.py [ROWS] [sizes...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
sizes = [int(x) for x in sys.argv[2:]] or [1, 4, 8, 9, 12, 16, 17, 24, 32, 33, 48, 64, 65, 128, 256, 512, 1024]
for n in sizes:
    R = max(1, rows // n)
    rng = np.random.default_rng(n)
    s = W.uniform(R, n, kind=W.FAIR_SHARE, seed=n)
    u = rng.random(R)
    s["kind"] = np.select([u < 0.4, u < 0.8, u < 0.9], [W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.STATIC],
                          W.NO_ALGORITHM).astype(np.int32)
    with Engine(0) as eng:
        eng.load(s)
        step = lambda: eng.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
        for _ in range(30):
            step()
        eng.sync()
        K = 200
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        eng.sync()
        dt = (time.perf_counter() - t0) / K
        eng.set_profiling(True)
        eng.reset_kernel_times()
        for _ in range(20):
            step()
        eng.sync()
        kt = {k: round(v[1] / max(v[0], 1) * 1e3, 2) for k, v in eng.kernel_times().items()}
        eng.set_profiling(False)
    N = R * n
    b = 28 * N + 97 * R
    print(json.dumps({"n": n, "resources": R, "leases": N, "us": round(dt * 1e6, 2), "GBs": round(b / dt / 1e9, 1),
                      "kernels": kt}), flush=True)
