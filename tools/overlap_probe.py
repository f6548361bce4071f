"""Do two work classes of one store overlap?  Stores of R resources with sizes drawn
from the given list (e.g. "2 3 4 5 6": small tiles + sub-wave groups), and the same
resources split into the two classes' stores alone; back-to-back writeback ticks.
usage: python tools/overlap_probe.py R size [size ...]"""
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

R = int(sys.argv[1])
choices = [int(x) for x in sys.argv[2:]]
rng = np.random.default_rng(5)
sizes = rng.choice(choices, R)


def store(sz):
    s = W.make_snapshot(sz, 0.0, 0.0, 1, W.NOW_NS + 3600 * W.NS, W.FAIR_SHARE, 1000.0)
    n = len(s["wants"])
    s["wants"] = rng.uniform(0.5, 1.5, n) * 1000.0 / np.repeat(sz, sz)
    s["has"] = np.minimum(s["wants"], 1000.0 / np.repeat(sz, sz))
    return W.add_store_sums(s)


def tick_us(s, K=300):
    with Engine(0) as eng:
        eng.load(s)
        step = lambda: eng.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
        for _ in range(50):
            step()
        eng.sync()
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
        info = eng.plan_info()
    return round(dt * 1e6, 2), kt, {k: info[k] for k in ("aux_own_queues", "stream_parts") if k in info}


out = {"sizes": choices, "R": R, "mixed": tick_us(store(sizes))}
lo, hi = sizes[sizes <= 4], sizes[sizes > 4]
if len(lo) and len(hi):
    out["le4_alone"] = tick_us(store(lo))
    out["gt4_alone"] = tick_us(store(hi))
print(json.dumps(out), flush=True)
