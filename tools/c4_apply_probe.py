"""configs[4]'s round without its tick: dm_store_apply alone per round (synchronous, as
the bench's step calls it), against the bare host-to-device copies of the same columns
(torch, one stream, page-locked), to see what the apply adds to PCIe time.
usage: python tools/c4_apply_probe.py [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
snap = bench.make_workload("c4", 0)
eng = Engine(0)
eng.load(snap)
step = bench.streaming_step(eng, snap, 0, 3 * rounds + 4)
for _ in range(2):
    step()
eng.sync()
out = {}
t0 = time.perf_counter()
for _ in range(rounds):
    step.apply_only()
eng.sync()
out["apply_ms"] = round((time.perf_counter() - t0) / rounds * 1e3, 3)
t0 = time.perf_counter()
for _ in range(rounds):
    step()
eng.sync()
out["step_ms"] = round((time.perf_counter() - t0) / rounds * 1e3, 3)
# the same bytes as bare copies: mask, packed wants, departures, arrivals (rows, wants, int32 subclients)
N = len(snap["wants"])
sizes = {"mask": N // 8, "wants": 8 * (N // 10), "gone": 8 * (N // 100), "new_rows": 8 * (N // 100),
         "new_wants": 8 * (N // 100), "new_sub": 4 * (N // 100)}
src = {k: torch.empty(v, dtype=torch.uint8).pin_memory() for k, v in sizes.items()}
dst = {k: torch.empty(v, dtype=torch.uint8, device="cuda") for k, v in sizes.items()}
s = torch.cuda.Stream()
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(rounds):
        with torch.cuda.stream(s):
            for k in sizes:
                dst[k].copy_(src[k], non_blocking=True)
        s.synchronize()
    out["bare_copies_ms"] = round((time.perf_counter() - t0) / rounds * 1e3, 3)
out["bytes_MB"] = round(sum(sizes.values()) / 1e6, 1)
eng.close()
print(json.dumps(out), flush=True)
