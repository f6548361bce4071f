"""The bench's bytes model and per-kernel units (CPU): what `roofline.achieved` and
`tick_hbm_frac` divide by."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402


def test_algorithmic_bytes_with_dense_rows():
    # 28 B per lease, 24 B for the rows of dense resources, 97 B per resource
    assert bench.algorithmic_bytes(1000, 10) == 28 * 1000 + 97 * 10
    assert bench.algorithmic_bytes(1000, 10, 1000) == 24 * 1000 + 97 * 10
    assert bench.algorithmic_bytes(1000, 10, 250.0) == 27 * 1000 + 97 * 10
    # C3: 100M leases in 100k resources, every resource dense after the first tick
    assert bench.algorithmic_bytes(100_000_000, 100_000, 100_000_000) == 2_409_700_000


def test_kernel_units_cover_every_row_once():
    sizes = np.array([0, 1, 8, 9, 16, 17, 32, 33, 64, 65, 128, 129, 256, 257, 512, 513, 1024, 1025, 2048, 2049,
                      4096, 4097, 9000])
    snap = W.make_snapshot(sizes, 1.0, 0.0, 1, W.NOW_NS + W.NS, W.FAIR_SHARE, 10.0)
    units = bench.kernel_units(snap)
    bins = ["small_packed", "sub8x2", "sub16x2", "sub16x4", "sub32x4", "wave64x4", "block128x4", "block128x8",
            "block256x8", "block512x8", "large_a"]
    assert sum(units[b][0] for b in bins) == int(sizes.sum())
    assert sum(units[b][1] for b in bins) == len(sizes)
    # the merged sub-wave launch covers exactly the five sub-wave bins
    sub = ["sub8x2", "sub16x2", "sub16x4", "sub32x4", "wave64x4"]
    assert units["subs_merged"] == (sum(units[b][0] for b in sub), sum(units[b][1] for b in sub))
    assert units["block128x8"] == (513 + 1024, 2)
