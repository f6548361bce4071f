"""Probe: does splitting one work class over two hardware queues hide the kernel's
ramp and tail?  One rank's configs[3] shard (N-way) as K engines over K contiguous
resource ranges, each on a CU-masked stream of its own (a hardware queue each), ticked
back to back; against one engine on one such stream.
  python tools/shard_split.py [N] [mK ...]   (m masked streams, j masked + joined every tick, p torch streams, o own streams; K engines)
"""
import ctypes
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


def masked():
    hip = ctypes.CDLL("libamdhip64.so")
    sp = ctypes.c_void_p()
    m = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(sp), 8, m) == 0
    return sp.value


def run(snap, mode, k, steps=300, warm=30):
    R = len(snap["seg_off"]) - 1
    cut = np.linspace(0, R, k + 1).astype(np.int64)
    engs = []
    for j in range(k):
        e = Engine(0)
        e.load(W.subset(snap, np.arange(cut[j], cut[j + 1])))
        if mode in ("m", "j"):
            e.set_stream(masked())
        elif mode == "p":
            e.set_stream(torch.cuda.Stream().cuda_stream)
        engs.append(e)
    tw = time.perf_counter()  # ~0.5 s of warm ticks (the first milliseconds run slow: bench.timed_steps)
    i = 0
    while time.perf_counter() - tw < 0.5 or i < warm:
        for e in engs:
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
        i += 1
        if i % 8 == 0:
            for e in engs:
                e.sync()
    for e in engs:
        e.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        for e in engs:
            e.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
        if mode == "j":  # every tick joined: each stream waits for the others' tick
            for a in engs:
                for b in engs:
                    if a is not b:
                        a.stream_wait(b.stream)
    for e in engs:
        e.sync()
    dt = (time.perf_counter() - t0) / steps * 1e6
    for e in engs:
        e.set_stream(None)
        e.close()
    return dt


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ks = sys.argv[2:] or ["m1", "m2", "o1", "o2", "p1", "p2"]  # m masked, p torch stream, o the engine's own
    torch.cuda.set_device(0)
    snap = bench.make_workload("c3", 0, n, "sharded")
    nb = len(snap["wants"]) * 24 + (len(snap["seg_off"]) - 1) * 97
    for k in ks:
        us = run(snap, k[0], int(k[1:]))
        print(f"shard {n}, {k} ({os.environ.get('GPU_MAX_HW_QUEUES', '-')} hw queues): {us:.2f} us per tick ({nb / us / 1e6:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
