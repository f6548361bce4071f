"""k_general timing: one 100k-row heterogeneous FairShare resource with 150 distinct
subclient counts, for library builds (e.g. the per-threshold-pass variant)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402
from test_general_gpu import hetero_snapshot  # noqa: E402

snap = hetero_snapshot(np.random.default_rng(5), [100_000], 150)
for lib in sys.argv[1:]:
    e = Engine(0, os.path.abspath(lib))
    e.load(snap)
    e.apportion(W.NOW_NS)
    e.set_profiling(True)
    e.reset_kernel_times()
    for _ in range(5):
        e.apportion(W.NOW_NS)
    kt = e.kernel_times()
    e.close()
    print(os.path.basename(lib), {k: round(ms / n * 1e3, 1) for k, (n, ms) in kt.items()}, "us per launch")
