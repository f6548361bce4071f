"""Cost of the hierarchy's root round on one GPU for G simulated servers (what an N-GPU
bench step adds besides the RCCL all-gather): dm_hier_root_tick over R resources with
a prefilled gathered buffer, timed with events over many rounds.

  python tools/hier_probe.py [--resources 100000] [--servers 1 2 4 8]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from doorman_amd import _lib  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402
from doorman_amd.hierarchy import root_snapshot  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resources", type=int, default=100_000)
    ap.add_argument("--servers", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--rounds", type=int, default=200)
    args = ap.parse_args()
    R = args.resources
    leaf_snap = W.make_snapshot(np.full(R, 4), 1.0, 0.0, 1, W.NOW_NS + 300 * W.NS, W.FAIR_SHARE, 1000.0)
    for G in args.servers:
        leaf, root = Engine(0), Engine(0)
        leaf.load(leaf_snap)
        root.load(root_snapshot(R, G, W.FAIR_SHARE, np.full(R, 1000.0 * G), lease_length_s=20))
        stream = torch.cuda.Stream()
        leaf.set_stream(stream.cuda_stream)
        root.set_stream(stream.cuda_stream)
        g = torch.empty((G * R, 2), dtype=torch.float64, device="cuda")
        g[:, 0] = 900.0  # SumWants
        g[:, 1] = torch.tensor([1000], dtype=torch.int64).view(torch.float64).item()  # Count bits
        L = root._L
        now = W.NOW_NS

        def rnd(t):
            _lib.check(L.dm_hier_root_tick(root._ctx, g.data_ptr(), G, int(now + t * W.NS), leaf._ctx, 0), root._ctx, L)

        for t in range(20):
            rnd(t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ext = torch.cuda.ExternalStream(stream.cuda_stream)
        e0.record(ext)
        for t in range(args.rounds):
            rnd(20 + t)
        e1.record(ext)
        torch.cuda.synchronize()
        print(f"G={G:2d} R={R}: {e0.elapsed_time(e1) * 1e3 / args.rounds:7.1f} us per root round "
              f"(k_hier_validate + k_hier_tick)", flush=True)
        leaf.close()
        root.close()


if __name__ == "__main__":
    main()
