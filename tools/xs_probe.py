"""Cost of a cross-stream dependency on this box (HIP events vs stream memory ops).

  python tools/xs_probe.py

Each case runs ~100 iterations of a ~100-us kernel (a torch add over 256 MB) and
reports the mean period per iteration minus the one-stream period:
  events:  A: kernel -> record e1; B: wait e1 -> kernel -> record e2; A: wait e2 -> ...
  stale:   A: kernel; wait on an event B recorded long ago (already complete at run time
           but not at enqueue time: B's kernel is short and early)
  value:   the same ping-pong with hipStreamWriteValue32 / hipStreamWaitValue32
"""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
hip.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
hipStreamWaitValueGte = 0


def timed(fn, iters=100):
    fn(5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(iters)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    dev = torch.device("cuda", 0)
    x = torch.ones(32 << 20, dtype=torch.float64, device=dev)
    y = torch.ones(32 << 20, dtype=torch.float64, device=dev)
    small = torch.ones(1024, device=dev)
    A, B = torch.cuda.Stream(), torch.cuda.Stream()

    def one(n):
        with torch.cuda.stream(A):
            for _ in range(n):
                x.add_(y)

    def events(n):
        for _ in range(n):
            e1 = torch.cuda.Event()
            with torch.cuda.stream(A):
                x.add_(y)
                e1.record(A)
            B.wait_event(e1)
            e2 = torch.cuda.Event()
            with torch.cuda.stream(B):
                small.add_(1.0)
                e2.record(B)
            A.wait_event(e2)

    def events_side(n):  # B waits on A each iteration, A never waits on B
        for _ in range(n):
            e1 = torch.cuda.Event()
            with torch.cuda.stream(A):
                x.add_(y)
                e1.record(A)
            B.wait_event(e1)
            with torch.cuda.stream(B):
                small.add_(1.0)

    flag = torch.zeros(64, dtype=torch.int32, device=dev)
    cnt = [0]

    def value(n):
        for _ in range(n):
            cnt[0] += 1
            v = cnt[0]
            with torch.cuda.stream(A):
                x.add_(y)
            rc = hip.hipStreamWriteValue32(A.cuda_stream, flag.data_ptr(), v, 0)
            rc |= hip.hipStreamWaitValue32(B.cuda_stream, flag.data_ptr(), v, hipStreamWaitValueGte, 0xFFFFFFFF)
            assert rc == 0, rc
            with torch.cuda.stream(B):
                small.add_(1.0)
            hip.hipStreamWriteValue32(B.cuda_stream, flag.data_ptr() + 4, v, 0)
            hip.hipStreamWaitValue32(A.cuda_stream, flag.data_ptr() + 4, v, hipStreamWaitValueGte, 0xFFFFFFFF)

    base = timed(one)
    print(f"one stream: {base:7.1f} us per iteration (kernel only)", flush=True)
    for name, fn in (("events ping-pong", events), ("events one-way", events_side), ("wait/write value", value)):
        t = timed(fn)
        print(f"{name:18s}: {t:7.1f} us per iteration, +{t - base:6.1f} over one stream", flush=True)


if __name__ == "__main__":
    main()
