"""C4 streaming step broken down: host-synchronous time of each store update call
and of the tick (one GPU), plus the H2D rate from page-locked memory.

  python tools/c4_probe.py [--steps 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import make_workload, streaming_step  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    snap = make_workload("c4", 0)
    eng = Engine(0)
    eng.load(snap)
    step = streaming_step(eng, snap, 0, args.steps + 2)
    # reach into the pre-generated batches through the closure
    it = step.__closure__[step.__code__.co_freevars.index("it")].cell_contents
    for k in range(args.steps + 2):
        mask, w, gone, new, nh, nw, ns, ne, t = next(it)
        ts = [time.perf_counter()]
        eng.update_wants_mask(mask, w)
        eng.sync()
        ts.append(time.perf_counter())
        eng.release(gone)
        eng.sync()
        ts.append(time.perf_counter())
        eng.upsert(new, nh, nw, ns, ne)
        eng.sync()
        ts.append(time.perf_counter())
        eng.apportion(t, writeback=True)
        ts.append(time.perf_counter())
        d = np.diff(ts) * 1e3
        mb = (mask.nbytes + w.nbytes) / 1e6
        print(f"step {k}: update_wants_mask {d[0]:.2f} ms ({len(w)} rows, {mb:.0f} MB -> {mb / d[0]:.1f} GB/s) "
              f"release {d[1]:.2f} ms ({len(gone)}) upsert {d[2]:.2f} ms ({len(new)}) tick {d[3]:.2f} ms", flush=True)
    n = 200 * 2 ** 20 // 8
    big = torch.empty(n, dtype=torch.float64).pin_memory()
    dst = torch.empty(n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(big, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"pinned H2D {n * 8 / dt / 1e9:.1f} GB/s")


if __name__ == "__main__":
    main()
