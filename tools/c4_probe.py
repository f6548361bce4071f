"""configs[4]: what a round's updates cost the next tick.  The bench's store and update
batches (bench.streaming_step), the tick's kernel time (HIP events) under variants:
  bench      the bench's step: apply (synchronous), tick (asynchronous), the next apply's
             copies overlapping the tick
  sync       the same, with a sync after each tick (no overlap with the next apply)
  none       no updates at all, synced ticks
  none_async no updates, back-to-back asynchronous ticks
  heater     the bench's step while a side stream keeps the GPU busy (one spinning
             kernel, torch.cuda._sleep): the clock state without the idle gaps, the store
             updates unchanged
  memheater  the same with 1-GiB device-to-device copies on the side stream instead
             (HBM traffic through the rounds)
usage: python tools/c4_probe.py [rounds] [variant ...]"""
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

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
variants = sys.argv[2:] or ["fresh", "none_async", "reloaded"]
snap = bench.make_workload("c4", 0)
out = {}
for variant in variants:
    eng = Engine(0)
    eng.load(snap)
    step = bench.streaming_step(eng, snap, 0, 2 * rounds + 8)
    if variant != "fresh":
        for _ in range(3):
            step()
        eng.sync()
        step.finish()
    if variant == "reloaded":  # the state after the rounds, loaded again into a fresh store
        st, rs = eng.read_store(), eng.resources(safe=False)
        s2 = dict(snap)
        s2.update(wants=st["wants"], has=st["has"], subclients=st["subclients"], expiry_ns=st["expiry_ns"],
                  agg_count=rs["count"], agg_sum_has=rs["sum_has"], agg_sum_wants=rs["sum_wants"])
        eng.close()
        eng = Engine(0)
        eng.load(s2)
    if variant in ("fresh", "reloaded"):
        for _ in range(3):
            eng.apportion(W.NOW_NS + 3 * 5 * W.NS, writeback=True)
    t = W.NOW_NS + 3 * 5 * W.NS
    heat = None
    if variant == "heater":  # one spinning kernel on a side stream through the rounds
        hs = torch.cuda.Stream()
        heat = True
        with torch.cuda.stream(hs):
            torch.cuda._sleep(int(2.4e9 * 0.005 * rounds))
    if variant == "memheater":  # HBM traffic on a side stream: 1 GiB device copies through the rounds
        hs = torch.cuda.Stream()
        a = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        heat = (a, b)
        with torch.cuda.stream(hs):
            for _ in range(rounds * 6):  # ~0.4 ms each at ~5 TB/s of read + write
                b.copy_(a)
    eng.set_profiling(True)
    eng.reset_kernel_times()
    t0 = time.perf_counter()
    for _ in range(rounds):
        if variant in ("bench", "heater", "memheater"):
            step()
        elif variant == "none":
            t += 5 * W.NS
            eng.apportion(t, writeback=True)
        elif variant in ("none_async", "fresh", "reloaded"):
            t += 5 * W.NS
            eng.apportion(t, writeback=True, asynchronous=True, defer_join=True)
        else:
            t = step.apply_only()
            eng.apportion(t, writeback=True)
    eng.sync()
    step.finish()
    if heat is not None:
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / rounds
    kt = {k: round(v[1] / max(v[0], 1) * 1e3, 2) for k, v in eng.kernel_times().items()}
    out[variant + ("" if variant not in out else "_2")] = {"round_ms": round(dt * 1e3, 3), "kernels": kt, "dense": eng.store_stats()["dense_leases"]}
    eng.close()
print(json.dumps(out), flush=True)
