"""H2D copy rate from page-locked memory: one copy vs two concurrent streams (probe)."""
import time
import torch

n = 200 * 2 ** 20 // 8
src = [torch.empty(n // 2, dtype=torch.float64).pin_memory() for _ in range(2)]
big = torch.empty(n, dtype=torch.float64).pin_memory()
dst = torch.empty(n, dtype=torch.float64, device="cuda")
pageable = torch.empty(n, dtype=torch.float64)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for name, fn in [
    ("pinned 1 copy", lambda: dst.copy_(big, non_blocking=True)),
    ("pageable 1 copy", lambda: dst.copy_(pageable, non_blocking=True)),
    ("pinned 2 streams", None),
]:
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if fn:
            fn()
        else:
            with torch.cuda.stream(s1):
                dst[: n // 2].copy_(src[0], non_blocking=True)
            with torch.cuda.stream(s2):
                dst[n // 2:].copy_(src[1], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"{name:20s} {n * 8 / dt / 1e9:6.1f} GB/s ({dt * 1e3:.2f} ms for {n * 8 / 1e6:.0f} MB)")
