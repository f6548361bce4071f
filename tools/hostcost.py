"""Host submission cost vs device time of one tick.

  python tools/hostcost.py --workload c2 [LIB.so ...]

Per library: host time to enqueue K asynchronous ticks (no sync), wall time per
tick including the final sync, and the stream time between a HIP event pair
around the K ticks.  Submission time close to wall time = host-bound tick.
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
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    snap = make_workload(args.workload, 0)
    for lib in args.libs or [None]:
        e = Engine(0, os.path.abspath(lib)) if lib else Engine(0)
        e.load(snap)
        for _ in range(200):
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
        e.sync()
        ext = torch.cuda.ExternalStream(e.stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(ext)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
        t1 = time.perf_counter()
        b.record(ext)
        e.sync()
        t2 = time.perf_counter()
        k = args.steps
        print(f"{os.path.basename(lib or 'in-tree'):24s} submit {(t1 - t0) / k * 1e6:8.1f} us/tick  "
              f"wall {(t2 - t0) / k * 1e6:8.1f} us/tick  stream {a.elapsed_time(b) / k * 1e3:8.1f} us/tick")
        e.close()


if __name__ == "__main__":
    main()
