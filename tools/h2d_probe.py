"""Host-to-device copy rate from page-locked memory: one stream vs several concurrent
streams (each its own part of the buffer), the configs[4] round's size (~150 MB) and
smaller pieces.  usage: python tools/h2d_probe.py"""
import json
import time

import torch


def rate(total, nstreams, pieces, reps=10):
    src = torch.empty(total, dtype=torch.uint8).pin_memory()
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    step = total // pieces
    for _ in range(2):
        for i in range(pieces):
            with torch.cuda.stream(streams[i % nstreams]):
                dst[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for i in range(pieces):
            with torch.cuda.stream(streams[i % nstreams]):
                dst[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step], non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return round(total / dt / 1e9, 2), round(dt * 1e3, 3)


out = []
for total in (150 << 20, 16 << 20):
    for ns, pieces in ((1, 1), (1, 4), (2, 2), (2, 4), (4, 4), (4, 8)):
        gbs, ms = rate(total, ns, pieces)
        out.append({"MB": total >> 20, "streams": ns, "pieces": pieces, "GB/s": gbs, "ms": ms})
        print(json.dumps(out[-1]), flush=True)
