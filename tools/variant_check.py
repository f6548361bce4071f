"""Parity of A/B library builds (tools/ab_libs/*.so) against the oracle before their
timings are trusted: the smoke snapshot (every dispatch bin), IEEE edge values,
heterogeneous subclients, recompute mode, three writeback ticks with lapses between
them, and C2's first tick on sampled resources.  Test infrastructure (uses oracle/).

  python tools/variant_check.py tools/ab_libs/x.so [...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402,F401

from doorman_amd import workloads as W  # noqa: E402
from doorman_amd.engine import Engine  # noqa: E402
from oracle import oracle as O  # noqa: E402
from parity_util import (assert_leases_match, assert_resources_match, binned_sizes, float_close,  # noqa: E402
                         row_capacity, snapshot_with_sizes)


def check(path):
    rng = np.random.default_rng(11)
    n = 0
    for variant in ("plain", "edge", "hetero", "recompute"):
        sizes = np.concatenate([binned_sizes(rng, per_bin=3), rng.integers(0, 9, 400), rng.integers(9, 257, 200)])
        snap = snapshot_with_sizes(rng, sizes, hetero=variant == "hetero", edge=variant == "edge")
        if variant == "recompute":  # the store's sums rebuilt from the rows (the oracle does the same)
            for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
                snap.pop(k)
        with Engine(0, path) as e:
            e.load(snap)
            e.apportion(W.NOW_NS, recompute=variant == "recompute")
            gets, exp = e.leases()
            res = e.resources()
        ref = O.apportion(snap, W.NOW_NS)
        assert_leases_match(snap, gets, exp, ref, f"{variant}")
        assert_resources_match(snap, res, ref, f"{variant}")
        n += 1
    # writeback ticks with lapses: the store against the oracle applied in order
    sizes = np.concatenate([rng.integers(0, 9, 3000), rng.integers(9, 257, 600), rng.integers(257, 600, 20)])
    snap = snapshot_with_sizes(rng, sizes, expired_frac=0.05)
    W.add_store_sums(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    with Engine(0, path) as e:
        e.load(snap)
        now = W.NOW_NS
        for t in range(4):
            now += int(rng.integers(0, 40)) * W.NS
            e.apportion(now, writeback=True, asynchronous=True, defer_join=True)
            ref = O.apportion(host, now)
            live = ref["expiry_ns"] != W.RELEASED
            host["has"] = np.where(live, ref["gets"], 0.0)
            host["wants"] = np.where(live, host["wants"], 0.0)
            host["subclients"] = np.where(live, host["subclients"], 0)
            host["expiry_ns"] = ref["expiry_ns"].copy()
            W.add_store_sums(host)
        e.sync()
        st = e.read_store()
        np.testing.assert_array_equal(st["expiry_ns"], host["expiry_ns"])
        np.testing.assert_array_equal(st["subclients"], host["subclients"])
        assert float_close(st["has"], host["has"], row_capacity(host)).all()
        np.testing.assert_array_equal(e.resources(safe=False)["count"], host["agg_count"])
    n += 1
    snap = W.c2()
    with Engine(0, path) as e:
        e.load(snap)
        e.apportion(W.NOW_NS)
        gets, exp = e.leases()
    pick = np.unique(np.concatenate([np.arange(0, 12), rng.choice(1_000_000, 2000, replace=False)]))
    sub = W.subset(snap, pick)
    ref = O.apportion(sub, W.NOW_NS)
    so = snap["seg_off"]
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in pick])
    assert_leases_match(sub, gets[rows], exp[rows], ref, "c2 sample")
    n += 1
    return n


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(f"{os.path.basename(p)}: {check(os.path.abspath(p))} checks against the oracle passed", flush=True)
