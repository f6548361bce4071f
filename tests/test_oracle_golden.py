"""Pins the CPU oracle against the reference's own known answers.

Vectors: tests/golden/reference_kats.json, transcribed from
go/server/doorman/{algorithm,store,server}_test.go and doc/*.md (each entry
cites file:line).  The reference itself (Go) cannot be built in this image —
no Go toolchain — so these fixtures are the pin.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from doorman_amd import workloads as W

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))
NOW = W.NOW_NS


@pytest.mark.parametrize("case", KATS["sequential"], ids=lambda c: c["name"])
def test_sequential_tables(case):
    """algorithm_test.go:34-62 testAlgorithm: sequential requests, one mutating store."""
    ids = {}
    for c in case["cases"]:
        ids.setdefault(c[0], len(ids))
    store = O.Store(len(ids))
    if case["preload"]:  # :37-44, lease 300 s, refresh 5 s
        for name, has, wants, _, sub in case["cases"]:
            store.assign(ids[name], 300, 5, has, wants, sub, NOW)
    for i, (name, has, wants, should_get, sub) in enumerate(case["cases"]):
        lease = O.algorithm(case["kind"], store, case["capacity"], ids[name], has, wants, sub, NOW)
        assert lease.has == should_get, f"case {i + 1}: {lease.has!r} != {should_get!r}"
        if case["respect_max"]:
            assert store.sum_has() <= case["capacity"]
    if "post" in case:
        assert store.sum_has() == case["post"]["sum_has"]


@pytest.mark.parametrize("case", KATS["snapshot"], ids=lambda c: c["name"])
@pytest.mark.parametrize("mode", ["literal", "closed"])
def test_snapshot_kats(case, mode):
    n = len(case["wants"])
    snap = W.make_snapshot([n], case["wants"], case["has"], case["sub"], NOW + 300 * W.NS, case["kind"],
                           case["capacity"])
    out = O.apportion(snap, NOW, mode)
    assert out["gets"].tolist() == case["gets"]
    if "doc_rounded" in case:
        np.testing.assert_allclose(out["gets"], case["doc_rounded"], rtol=1e-9)


def test_store_kat():
    """store_test.go:22-77 (the 10 s sleep becomes a frozen clock step)."""
    k = KATS["store"]
    ids = {"a": 0, "b": 1, "c": 2}
    s = O.Store(3)
    for name, lease_s, ref_s, has, wants, sub in k["assign"]:
        s.assign(ids[name], lease_s, ref_s, has, wants, sub, NOW)
    a = k["after_assign"]
    assert (s.sum_has(), s.sum_wants(), s.get(0).has, s.count()) == (a["sum_has"], a["sum_wants"], a["get_a_has"],
                                                                     a["count"])
    s.clean(NOW + k["clean_after_s"] * W.NS + 1)
    c = k["after_clean"]
    assert (s.sum_has(), s.sum_wants(), s.get(0).is_zero()) == (c["sum_has"], c["sum_wants"], c["a_is_zero"])
    s.release(ids[k["release"]])
    assert s.get(2).is_zero()
    r = k["after_release"]
    assert (s.sum_has(), s.sum_wants(), s.count()) == (r["sum_has"], r["sum_wants"], r["count"])


def test_store_clean_is_strict_after():
    """store.go:174 when.After(lease.Expiry): a lease expiring exactly now survives."""
    s = O.Store(2)
    s.assign(0, 10, 1, 1.0, 1.0, 1, NOW)
    assert s.clean(NOW + 10 * W.NS) == 0
    assert s.clean(NOW + 10 * W.NS + 1) == 1


def test_lease_length_kat():
    k = KATS["lease_length"]
    s = O.Store(1)
    lease = O.algorithm(k["kind"], s, k["capacity"], 0, 0, k["wants"], k["sub"], NOW, k["lease_length"],
                        k["refresh_interval"])
    assert lease.expiry_ns // W.NS - NOW // W.NS == k["expiry_minus_now_s"]
    assert lease.refresh_ns == k["refresh_s"] * W.NS


def _cfg(case, master_at, kind=None):
    lmd = case["learning_mode_duration"]
    dur = case["lease_length"] if lmd is None else lmd  # resource.go:157-161
    learning_end = master_at + dur * W.NS if dur > 0 else 0  # server.go:173-179 (time.Unix(0,0))
    return O.make_cfg(1, kind=case["kind"] if kind is None else kind, capacity=case["capacity"],
                      lease_length_s=case["lease_length"], refresh_interval_s=case["refresh_interval"],
                      learning_end_ns=learning_end)[0]


@pytest.mark.parametrize("case", KATS["server"], ids=lambda c: c["name"])
def test_server_kats(case):
    master_at = NOW - W.NS // 2
    if "bands" in case:
        wants = [b[0] for b in case["bands"]]
        nums = [b[1] for b in case["bands"]]
        if "error" in case:
            with pytest.raises(ValueError):
                O.aggregate_bands(wants, nums)
            return
        wt, st = O.aggregate_bands(wants, nums)
        lease = O.decide(O.Store(1), _cfg(case, master_at), 0, case["has"], wt, st, NOW)
        assert lease.has == case["gets"]
        return
    store, cfg = O.Store(1), _cfg(case, master_at)
    if "release" in case:  # TestReleaseCapacity: a lease, then ReleaseCapacity (server.go:668-714)
        rel = case["release"]
        O.decide(store, cfg, 0, rel["request"]["has"], rel["request"]["wants"], 1, NOW)
        store.release(0)  # "resource"; "nonexisting_resource" is unknown and ignored (:705-710)
        assert store.sum_has() == rel["post_sum_has"]
        return
    for step in case["steps"]:
        if step.get("new_resource"):
            store, cfg = O.Store(1), _cfg(case, NOW - step["age_s"] * W.NS)
        if step.get("after_reload"):
            # LoadConfig swaps the template but keeps learningModeEndTime (resource.go:117-125)
            rl = dict(case["reload"])
            new = _cfg({**rl, "learning_mode_duration": rl["learning_mode_duration"]}, master_at)
            new["learning_end_ns"] = cfg["learning_end_ns"]
            cfg = new
        lease = O.decide(store, cfg, 0, step["has"], step["wants"], 1, NOW)
        assert lease.has == step["gets"], step


@pytest.mark.parametrize("seed", range(30))
def test_closed_form_equals_literal(seed):
    """the closed form is bit-identical to the literal restatement
    (same row order), including heterogeneous subclients, expiries, learning mode,
    parent expiry and IEEE edge values."""
    rng = np.random.default_rng(seed)
    snap = W.random_snapshot(rng, 6, 40, hetero=bool(seed % 2), edge=seed % 3 == 0)
    if seed % 4 == 0:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            snap.pop(k)
    a = O.apportion(snap, NOW, "literal")
    b = O.apportion(snap, NOW, "closed")
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.parametrize("variant", ["uniform", "hetero", "edge", "hetero_edge"])
def test_closed_form_equals_literal_large_resources(variant):
    """The same identity on resources of 1k-5k rows (every GPU parity test compares
    against the closed form at up to 1M rows per resource): FairShare and
    ProportionalShare with contention, heterogeneous subclients and IEEE edge values."""
    from parity_util import snapshot_with_sizes
    rng = np.random.default_rng(["uniform", "hetero", "edge", "hetero_edge"].index(variant) + 40)
    sizes = np.asarray([1000, 1800, 2500, 5000], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=(2, 3), hetero="hetero" in variant, edge="edge" in variant,
                               learning_frac=0.0, parent_expired_frac=0.0)
    snap["kind"] = np.asarray([2, 3, 3, 3], dtype=np.int32)
    a = O.apportion(snap, NOW, "literal")
    b = O.apportion(snap, NOW, "closed")
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_threaded_closed_form_matches():
    """The OpenMP comparator (bench.py cpu_baseline 'closed_mt') gives the same bits."""
    rng = np.random.default_rng(7)
    snap = W.random_snapshot(rng, 300, 40, hetero=True, edge=True)
    a = O.apportion(snap, NOW, "closed")
    b = O.apportion(snap, NOW, "closed", threads=4)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_unknown_kind_is_an_error():
    snap = W.make_snapshot([2], [1, 2], [0, 0], 1, NOW + W.NS, 7, 10.0)
    with pytest.raises(ValueError):
        O.apportion(snap, NOW, "closed")


@pytest.mark.parametrize("case", [c for c in KATS["server"] if "error" not in c and "release" not in c],
                         ids=lambda c: c["name"])
def test_server_kats_as_one_row_snapshots(case):
    """For a single client, Decide on an empty store (the reference's first request)
    and the snapshot tick of a store holding only that client agree: count,
    unused capacity, SumWants test and Learn all coincide.  This is what lets the
    GPU tests replay these KATs through dm_apportion (test_parity_gpu.py)."""
    for snap, expect in server_kat_snapshots(case):
        assert O.apportion(snap, NOW)["gets"][0] == expect
        assert O.apportion(snap, NOW, "literal")["gets"][0] == expect


def server_kat_snapshots(case):
    """(one-row snapshot, expected gets) for every step of a server KAT."""
    master_at = NOW - W.NS // 2
    out = []
    if "bands" in case:
        wt, st = O.aggregate_bands([b[0] for b in case["bands"]], [b[1] for b in case["bands"]])
        cfg = _cfg(case, master_at)
        out.append((W.make_snapshot([1], [wt], [case["has"]], [st], [NOW + W.NS], cfg["kind"], cfg["capacity"],
                                    cfg["lease_length_s"], cfg["refresh_interval_s"], cfg["learning_end_ns"]),
                    case["gets"]))
        return out
    cfg = _cfg(case, master_at)
    for step in case["steps"]:
        if step.get("new_resource"):
            cfg = _cfg(case, NOW - step["age_s"] * W.NS)
        if step.get("after_reload"):
            new = _cfg(dict(case["reload"]), master_at)
            new["learning_end_ns"] = cfg["learning_end_ns"]
            cfg = new
        out.append((W.make_snapshot([1], [step["wants"]], [step["has"]], [1], [NOW + W.NS], cfg["kind"],
                                    cfg["capacity"], cfg["lease_length_s"], cfg["refresh_interval_s"],
                                    cfg["learning_end_ns"]), step["gets"]))
    return out


@pytest.mark.parametrize("case", KATS["hierarchy"], ids=lambda c: c["name"])
def test_hierarchy_kat_model(case):
    """server_test.go:574-658 replayed on the reference model of the hierarchy
    (tests/hier_model.py): 0 before the intermediate's first exchange with the root,
    the full capacity after it."""
    import hier_model as M
    rt, it, band = case["root"], case["intermediate_default"], case["band"]
    root_cfg = {"kind": [rt["kind"]], "capacity": [rt["capacity"]], "lease_length_s": [rt["lease_length"]],
                "refresh_interval_s": [rt["refresh_interval"]], "learning_end_ns": [W.INT64_MIN],
                "parent_expiry_ns": [W.INT64_MAX], "safe_capacity": [np.nan]}
    leaf_cfg = {"kind": [it["kind"]], "capacity": [float(it["capacity"])], "lease_length_s": [it["lease_length"]],
                "refresh_interval_s": [it["refresh_interval"]], "learning_end_ns": [W.INT64_MIN],
                "parent_expiry_ns": [W.INT64_MAX], "safe_capacity": [float(it["safe_capacity"])]}
    leaf = O.Store(1)
    # the downstream server's band reaches the intermediate before its first exchange
    lease = O.decide(leaf, M.cfg_table(leaf_cfg)[0], 0, 0.0, band["wants"], band["num_clients"], NOW)
    assert lease.has == case["gets_before_exchange"]
    root = M.Root(root_cfg, 1)
    req = M.server_request([leaf.sum_wants()], [leaf.count()])
    resp = root.round(NOW, [req])
    leaf_cfg = M.leaf_templates(leaf_cfg, 0, resp, root.cfg)
    lease = O.decide(leaf, M.cfg_table(leaf_cfg)[0], 0, 0.0, band["wants"], band["num_clients"], NOW + W.NS)
    assert lease.has == case["gets_after_exchange"]
