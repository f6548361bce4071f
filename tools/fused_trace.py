"""Per-chunk timestamps of the one-launch large path (a tracing build made with
tools/mkvariant.sh; exports dm_debug_trace): C2's large resources, one tick after
warm-up ticks.  Writes gpurun_out/fused_trace.npz for offline analysis."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    lib = os.path.abspath(sys.argv[1])
    snap = W.c2()
    if "--all" not in sys.argv:
        sizes = np.diff(snap["seg_off"])
        snap = W.subset(snap, np.flatnonzero(sizes > 4096))
    e = Engine(0, lib)
    e.set_large_path(fused=True)
    e.load(snap)
    info = e.plan_info()
    for _ in range(5):
        e.apportion(W.NOW_NS, writeback=True)
    e.apportion(W.NOW_NS, writeback=True)
    n = info["fused_chunks"]
    buf = np.zeros(n * 8, dtype=np.uint64)
    L = ctypes.CDLL(lib)
    rc = L.dm_debug_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int(n))
    assert rc == 0, rc
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez("gpurun_out/fused_trace.npz", trace=buf.reshape(n, 8), sizes=np.diff(snap["seg_off"]))
    t = buf.reshape(n, 8).astype(np.int64)
    t0 = t[:, 0].min()
    print("span us", (t[:, 5].max() - t0) / 100.0, "chunks", n, info)
    e.close()


if __name__ == "__main__":
    main()
