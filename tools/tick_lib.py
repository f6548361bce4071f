"""Writeback ticks of one workload through one library build, for rocprofv3 runs
that compare builds (tools/mix_ab.sh):

  python tools/tick_lib.py --workload c3 --steps 10 LIB.so
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import make_workload  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    e = Engine(0, os.path.abspath(args.lib))
    e.load(make_workload(args.workload, 0))
    for _ in range(3 + args.steps):
        e.apportion(W.NOW_NS, writeback=True)
    torch.cuda.synchronize()
    e.close()


if __name__ == "__main__":
    main()
