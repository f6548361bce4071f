"""configs[2]'s tick after the host process created K hardware queues of its own first
(a host that embeds the library owns streams too).
usage: python tools/queue_probe.py K [torch|masked] [steps]
  torch:  K torch streams (torch.cuda.Stream), created before the engine
  masked: K CU-masked HIP streams (a hardware queue each), created before the engine
Prints one JSON line: the tick's us per step and the per-class event times."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

K = int(sys.argv[1])
how = sys.argv[2] if len(sys.argv) > 2 else "torch"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 400
torch.cuda.set_device(0)
keep = []
if how == "torch":
    for _ in range(K):
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            torch.zeros(16, device="cuda").add_(1)  # the stream is used, its queue exists
        keep.append(s)
else:
    hip = ctypes.CDLL("libamdhip64.so")
    mask = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
    for _ in range(K):
        st = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), 8, mask)
        assert rc == 0, rc
        keep.append(st)
torch.cuda.synchronize()

import bench  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402

snap = bench.make_workload("c2", 0)
with Engine(0) as eng:
    eng.load(snap)
    step = lambda: eng.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)  # noqa: E731
    for _ in range(2000):
        step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    eng.set_profiling(True)
    eng.reset_kernel_times()
    for _ in range(50):
        step()
    eng.sync()
    kt = {k: round(v[1] / max(v[0], 1) * 1e3, 2) for k, v in eng.kernel_times().items()}
    info = eng.plan_info()
print(json.dumps({"extra_queues": K, "how": how, "us": round(dt * 1e6, 2), "kernels": kt,
                  "calibrated_perm": info.get("queue_perm")}), flush=True)
