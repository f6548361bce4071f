"""Probe: the C2 tick in a process that first ran other contexts (bench.py's default
run measures configs[2] after configs[3] and configs[1]).  Prelude steps, in order:
  c1     a C1 engine: load, 60 ticks, close
  c3     a C3 engine (100M leases, no exchange): load, 20 ticks, close
  hier   configs[3]'s leaf + root with the pipelined exchange: 20 steps, close
  alloc  torch allocates and frees 4 GB of device memory
  ctx    an engine created and closed, nothing loaded
  c1keep a C1 engine loaded and ticked, kept open while C2 runs
then C2: load, bench.timed_steps (50 steps), print the tick time.
  python tools/c2_after.py [c1] [c3] [hier] [alloc]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


LIB = os.environ.get("DM_LIB") or None  # a tools/ab_libs variant


def ticks(e, n):
    for _ in range(n):
        e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
    e.sync()


def main():
    torch.cuda.set_device(0)
    keep = []
    for step in sys.argv[1:]:
        t0 = time.perf_counter()
        if step == "ctx":
            Engine(0, LIB).close()
        elif step == "c1keep":
            e = Engine(0, LIB)
            e.load(bench.make_workload("c1", 0))
            ticks(e, 60)
            keep.append(e)
        elif step in ("c1", "c3"):
            e = Engine(0, LIB)
            e.load(bench.make_workload(step, 0))
            ticks(e, 60 if step == "c1" else 20)
            e.close()
        elif step == "hier":
            from doorman_amd.hierarchy import HierarchicalTick, root_snapshot
            snap = bench.make_workload("c3", 0, 1, "sharded")
            leaf, root = Engine(0, LIB), Engine(0, LIB)
            leaf.load(snap)
            root.load(root_snapshot(bench.C3_R, 1, W.FAIR_SHARE, 1000.0, lease_length_s=20))
            ht = HierarchicalTick(torch, leaf, root, bench.C3_R, 1, 0, None, shard_lo=bench.c3_bounds(1),
                                  pipelined=True, native="local")
            for _ in range(20):
                ht.tick(W.NOW_NS, asynchronous=True)
            ht.sync()
            del ht
            leaf.close()
            root.close()
        elif step == "alloc":
            x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
            x.fill_(1)
            torch.cuda.synchronize()
            del x
            torch.cuda.empty_cache()
        print(f"prelude {step}: {time.perf_counter() - t0:.1f} s", flush=True)
    snap = bench.make_workload("c2", 0)
    e = Engine(0, LIB)
    e.load(snap)
    st = lambda: e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
    r = bench.timed_steps(torch, e, st, 50, 10, lambda what, v: v)
    print(f"{os.path.basename(LIB or 'prod')} after {' '.join(sys.argv[1:]) or '(nothing)'}: C2 {r['elapsed'] / 50 * 1e6:.1f} us per tick, "
          f"enqueue {r['host_enqueue_s'] / 50 * 1e6:.1f} us, plan {e.plan_info().get('aux_own_queues')}", flush=True)
    e.close()


if __name__ == "__main__":
    main()
