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
    bins = ["small_tiles", "sub8x2", "sub16x2", "sub16x4", "sub32x4", "wave64x4", "block128x4", "block128x8",
            "block256x8", "block2k4k", "large_a"]
    assert sum(units[b][0] for b in bins) == int(sizes.sum())
    assert sum(units[b][1] for b in bins) == len(sizes)
    # the merged sub-wave launch covers exactly the five sub-wave bins
    sub = ["sub8x2", "sub16x2", "sub16x4", "sub32x4", "wave64x4"]
    assert units["subs_merged"] == (sum(units[b][0] for b in sub), sum(units[b][1] for b in sub))
    assert units["block128x8"] == (513 + 1024, 2)


def test_every_kernel_class_has_units():
    """Every class dm_kernel_times can report (the library's own list, no GPU needed) has
    a units entry, so the roofline never falls back to whole-snapshot bytes; an unknown
    name raises."""
    from doorman_amd import _lib
    sizes = np.array([1, 9, 300, 5000])
    snap = W.make_snapshot(sizes, 1.0, 0.0, 1, W.NOW_NS + W.NS, W.FAIR_SHARE, 10.0)
    units = bench.kernel_units(snap)
    names = _lib.kernel_class_names()
    assert "large_spec" in names and "large_redo" in names and "hier_gather" in names
    missing = [n for n in names if n not in units]
    assert not missing, missing
    run = {"ktimes": {"no_such_kernel": (1, 1.0)}, "stream_ms": 1.0}
    try:
        bench.roofline_of("c2", snap, run, 1, False)
    except KeyError:
        pass
    else:
        raise AssertionError("an unknown kernel class must raise")


def test_large_spec_roofline_counts_the_large_class_only():
    """C2's speculative chain: the roofline divides by the > 4096-row class's bytes (24 B
    per lease: the steady tick reads no subclients column), not the whole snapshot's
    (round 4's line reported 3x the real fraction)."""
    snap = bench.make_workload("c2", 0)
    sizes = np.diff(snap["seg_off"])
    big = sizes > 4096
    run = {"ktimes": {"large_spec": (10, 1.0), "subs_merged": (10, 0.5)}, "stream_ms": 1.0, "dense_frac": 1.0}
    r = bench.roofline_of("c2", snap, run, 10, False)
    assert r["kernel"] == "large_spec"
    assert r["leases_per_launch"] == int(sizes[big].sum()) and r["resources_per_launch"] == int(big.sum())
    assert r["algorithmic_bytes_per_launch"] == 24 * int(sizes[big].sum()) + 97 * int(big.sum())
    # C2's large class: 6.08M leases in 244 resources
    assert 6.0e6 < r["leases_per_launch"] < 6.2e6 and r["resources_per_launch"] == 244


def test_stream_parts_roofline_is_per_tick():
    """C1's one bin in two stream parts: two concurrent launches per tick, each over half
    the bin.  The roofline takes the whole bin's bytes over the tick's time (the timed
    region's events), and the PMC traffic (recorded per launch) times the parts."""
    snap = bench.make_workload("c1", 0)
    steps = 10
    run = {"ktimes": {"block128x8_dense": (2 * steps, 0.6)}, "stream_ms": 0.4, "dense_frac": 1.0, "parts": 2}
    r = bench.roofline_of("c1", snap, run, steps, True)
    N, R = len(snap["wants"]), len(snap["seg_off"]) - 1
    assert r["stream_parts"] == 2 and r["leases_per_launch"] == N
    assert r["avg_launch_us"] == 40.0  # 0.4 ms over 10 ticks, not 0.6 ms over 20 launches
    assert abs(r["achieved"] - (24 * N + 97 * R) / 40e-6 / 1e9) < 0.1
    if r["traffic"] is not None:
        import json
        per_launch = json.load(open(os.path.join(ROOT, "profiles", "pmc_c1.json")))["block128x8_dense"]
        assert r["traffic"] == 2 * per_launch["hbm_bytes_per_launch"]


def test_self_check_root_round_matches_the_reference_model():
    """bench.root_round_one (the N > 1 exchange self-check's restatement of the sharded
    root round, one row per resource) against the hierarchy model (tests/hier_model.py:
    the oracle's literal Decide) over rounds with every kind, learning resources, an
    expired parent, rows that lapse between rounds and resources left unrequested:
    templates and grants bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import hier_model as M
    rng = np.random.default_rng(77)
    R = 200
    now = W.NOW_NS
    cfg = {"kind": rng.integers(0, 4, R).astype(np.int32), "capacity": rng.choice([0.0, 5.0, 300.0, 1000.0], R),
           "lease_length_s": rng.choice([1, 10, 20], R).astype(np.int64),
           "refresh_interval_s": rng.choice([1, 5], R).astype(np.int64),
           "learning_end_ns": np.where(rng.random(R) < 0.1, now + 3 * W.NS, W.INT64_MIN).astype(np.int64),
           "parent_expiry_ns": np.where(rng.random(R) < 0.1, now + 2 * W.NS, W.INT64_MAX).astype(np.int64),
           "safe_capacity": np.where(rng.random(R) < 0.3, 4.5, np.nan)}
    model = M.Root(cfg, 1)
    cols = [cfg[f] for f in ("kind", "capacity", "lease_length_s", "refresh_interval_s", "learning_end_ns",
                             "parent_expiry_ns", "safe_capacity")]
    checked = 0
    for t in range(8):
        now += int(rng.choice([0, 1, 4, 12])) * W.NS
        sw = np.where(rng.random(R) < 0.8, rng.uniform(0.0, 2000.0, R), 0.0)
        cnt = rng.integers(1, 6, R)
        rows, sums = model.rows(), model.sums()
        req = M.server_request(sw, cnt)
        resp = model.round(now, [req])
        tpl = M.leaf_templates(M.default_config(R), 0, resp, model.cfg)
        for r in range(R):
            got = bench.root_round_one(now, [c[r] for c in cols],
                                       (rows["wants"][r], rows["has"][r], rows["subclients"][r], rows["expiry_ns"][r]),
                                       (sums["count"][r], sums["sum_has"][r], sums["sum_wants"][r]), 0, sw[r],
                                       int(cnt[r]))
            want = tuple(np.asarray(tpl[f][r]).item() for f in bench._TPL_FIELDS)
            assert np.asarray(got[0], dtype=object).tolist() == list(want) or all(
                np.float64(a).tobytes() == np.float64(b).tobytes() for a, b in zip(got[0], want)), (t, r, got, want)
            if (0, r) in resp:
                assert np.float64(got[1]).tobytes() == np.float64(resp[(0, r)].has).tobytes(), (t, r)
            checked += 1
    assert checked == 8 * R
    assert bench.root_round_one(now, [c[0] for c in cols], (0.0, 0.0, 0, W.RELEASED), (0, 0.0, 0.0), 1, 5.0, 1) is None


def test_l3_resident_flag_c1_not_c3():
    """A tick whose distinct bytes fit the 256 MiB Infinity Cache (C1: 10M leases written
    in place, 160-200 MB) is flagged l3_resident and reports no HBM fraction; C3 (100M
    leases, 2.4 GB per tick) and C2 (14M leases with an alternate gets column) are HBM
    lines."""
    c1 = {"seg_off": np.arange(0, 10_000_001, 1000, dtype=np.int64)}
    c3 = {"seg_off": np.arange(0, 100_000_001, 1000, dtype=np.int64)}
    c2 = {"seg_off": np.concatenate([[0], np.cumsum(W.zipf_sizes())])}
    f1 = bench.tick_footprint_bytes(c1, 10_000_000)
    assert f1["l3_resident"] and not f1["alternate_gets_column"] and f1["tick_footprint_bytes"] < 256 << 20
    assert bench.tick_footprint_bytes(c1, 0)["l3_resident"]  # 200 MB even with the subclients column
    assert not bench.tick_footprint_bytes(c3, 100_000_000)["l3_resident"]
    f2 = bench.tick_footprint_bytes(c2, 0)
    assert f2["alternate_gets_column"] and not f2["l3_resident"]
    # the fractions: C1's goes to tick_frac_l3, C3's stays an HBM fraction
    t1 = bench.tick_fracs(c1, 1.0, 40e-6)
    assert t1["tick_hbm_frac"] is None and t1["tick_frac_l3"] > 0
    t3 = bench.tick_fracs(c3, 1.0, 440e-6)
    assert t3["tick_frac_l3"] is None and abs(t3["tick_hbm_frac"] - 2_409_700_000 / 440e-6 / 8e12) < 1e-4
    snap = bench.make_workload("c1", 0)
    run = {"ktimes": {"block128x8_dense": (20, 0.6)}, "stream_ms": 0.4, "dense_frac": 1.0, "parts": 2}
    r = bench.roofline_of("c1", snap, run, 10, True)
    assert r["l3_resident"] and r["frac"] is None and r["frac_l3"] > 0 and r["frac_of_copy_ceiling"] is None
