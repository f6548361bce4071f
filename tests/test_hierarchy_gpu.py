"""The intermediate-server hierarchy on one GPU (dm_hier_root_tick), against the
reference model of tests/hier_model.py -- restated from server.go:227-323,
:822-901 and resource.go:62-70,117-125, not from the kernels.

G servers each publish their store totals, run the root's round on their own
copy of the root store (as every rank of a node does) and load their new
templates, then tick their leaf store.  Per round:
  * every root copy equals the model's root stores bit for bit (rows and running
    sums: the kernel decides the servers' requests one after another in server
    order, each seeing the Assigns before it, as the root's res.mu serialises
    GetServerCapacity calls, and walks the rows in the oracle's order);
  * every leaf's configuration equals the model's templates bit for bit (grant,
    parent expiry in Unix seconds, the root's algorithm and safe capacity, or the
    "*" default for resources it did not request; learning end kept);
  * every leaf's leases match the oracle on that leaf's store and templates.
"""
import json
import os

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
import hier_model as M
from parity_util import assert_leases_match

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS
HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))


def root_config(R, rng):
    """The root's own resource configuration: every kind, learning mode on a few,
    configured and unset safe capacities, several lease lengths."""
    kind = rng.choice([W.FAIR_SHARE, W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.STATIC, W.NO_ALGORITHM], R).astype(np.int32)
    return {"kind": kind, "capacity": rng.choice([100.0, 1000.0, 2500.5], R),
            "lease_length_s": rng.choice([7, 20, 60], R).astype(np.int64),
            "refresh_interval_s": rng.choice([1, 5], R).astype(np.int64),
            "learning_end_ns": np.where(rng.random(R) < 0.1, NOW + 3 * W.NS, W.INT64_MIN).astype(np.int64),
            "parent_expiry_ns": np.full(R, W.INT64_MAX, np.int64),
            "safe_capacity": np.where(rng.random(R) < 0.5, np.nan, rng.uniform(1, 9, R))}


def root_engine(cfg, G):
    from doorman_amd.engine import Engine
    R = len(cfg["kind"])
    N = R * G
    snap = W.make_snapshot(np.full(R, G), np.zeros(N), np.zeros(N), np.zeros(N, np.int64), np.full(N, W.RELEASED),
                           cfg["kind"], cfg["capacity"], cfg["lease_length_s"], cfg["refresh_interval_s"],
                           cfg["learning_end_ns"], cfg["parent_expiry_ns"], cfg["safe_capacity"])
    e = Engine(0)
    e.load(snap)
    return e


def leaf_snapshot(e, cfg):
    """The leaf's store as the device holds it (rows + running sums) under `cfg`."""
    st = e.read_store()
    res = e.resources(safe=False)
    R = e.n_resources
    snap = dict(cfg)
    snap.update({"wants": st["wants"], "has": st["has"], "subclients": st["subclients"], "expiry_ns": st["expiry_ns"],
                 "agg_count": res["count"], "agg_sum_has": res["sum_has"], "agg_sum_wants": res["sum_wants"]})
    snap["seg_off"] = e.seg_off
    assert len(snap["seg_off"]) == R + 1
    return snap


def assert_cfg_equal(got, want, label):
    for k in W.CFG_FIELDS:
        a, b = np.asarray(got[k]), np.asarray(want[k])
        same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
        assert same.all(), f"{label}: template field {k} differs at resources {np.flatnonzero(~same)[:8].tolist()}: " \
                           f"{a[~same][:4].tolist()} vs {b[~same][:4].tolist()}"


def assert_root_equal(e, model, label):
    st, res = e.read_store(), e.resources(safe=False)
    rows, sums = model.rows(), model.sums()
    for k in ("has", "wants", "subclients", "expiry_ns"):
        assert st[k].tobytes() == rows[k].tobytes(), f"{label}: root {k} rows " \
            f"{np.flatnonzero(st[k] != rows[k])[:8].tolist()}"
    for k in ("count", "sum_has", "sum_wants"):
        assert res[k].tobytes() == sums[k].tobytes(), f"{label}: root running {k}"


def published(gathered, G, R, stride=None):
    """Every server's published block (dm_publish_totals): (SumWants, Count, flags)."""
    S = R + 1 if stride is None else stride
    rec = gathered.cpu().numpy()
    out = []
    for g in range(G):
        b = rec[g * S:g * S + 1 + R]
        f = int(b[0, 0:1].view(np.uint64)[0])  # the OR of record 0's two flags words (DevParams::pub_word)
        out.append((b[1:, 0].copy(), b[1:, 1].copy().view(np.int64), (f & 0xFFFFFFFF) | (f >> 32)))
    return out


def blocks(sum_wants, counts, flags=None):
    """A gathered buffer built on the host: one block per server, record 0 = flags."""
    G, R = sum_wants.shape
    rec = np.zeros((G, R + 1, 2))
    rec[:, 1:, 0] = sum_wants
    rec[:, 1:, 1] = np.ascontiguousarray(counts, dtype=np.int64).view(np.float64)
    if flags is not None:
        rec[:, 0, 0] = np.asarray(flags, dtype=np.int64).view(np.float64)
    return rec.reshape(G * (R + 1), 2)


def model_flags(sum_wants, counts):
    """The validation dm_publish_totals attaches (server.go:863-866 + the 32-bit column)."""
    band = sum_wants > 0
    return (np.any(band & (counts < 1)) * 1) | (np.any(band & (counts > 2**31 - 2)) * 2)


def exchange_all(L, roots, leaves, gathered, G, now):
    from doorman_amd import _lib
    for g in range(G):
        _lib.check(L.dm_hier_root_tick(roots[g]._ctx, gathered.data_ptr(), G, now, leaves[g]._ctx, g), roots[g]._ctx)
    for e in roots + leaves:
        e.sync()


@pytest.mark.parametrize("clients", [0, 600])
@pytest.mark.parametrize("G", [1, 2, 3, 8, 20])
def test_hierarchy_rounds_match_the_reference_model(G, clients):
    """clients = 0: 3-119 clients per leaf resource; 600: every leaf resource on the
    128-thread kernels, dense (and split) from its second writeback tick."""
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    L = _lib.lib()
    R = 48
    rng = np.random.default_rng(G)
    rcfg = root_config(R, rng)
    leaves, tpl = [], []
    for g in range(G):
        s = W.uniform(R, clients or int(rng.integers(3, 120)), kind=W.FAIR_SHARE, seed=10 * G + g,
                      capacity=1000.0)
        s["wants"] *= rng.uniform(0.2, 3.0)  # servers differ in appetite
        W.add_store_sums(s)
        cfg = M.default_config(R, np.where(rng.random(R) < 0.1, NOW + 2 * W.NS, W.INT64_MIN))
        e = Engine(0)
        e.load(M.with_config(s, cfg))
        leaves.append(e)
        tpl.append(cfg)
    roots = [root_engine(rcfg, G) for _ in range(G)]
    model = M.Root(rcfg, G)
    gathered = torch.zeros((G * (R + 1), 2), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream, written on the context's
    for t, now in enumerate([NOW, NOW + 5 * W.NS, NOW + 9 * W.NS, NOW + 40 * W.NS]):
        if t == 2 and G > 1:  # server 1 stops asking for a quarter of the resources
            so = leaves[1].seg_off
            rows = np.arange(so[0], so[R // 4])
            leaves[1].update_wants(rows, np.zeros(len(rows)))
        for g in range(G):
            leaves[g].publish_totals(gathered[g * (R + 1):(g + 1) * (R + 1)].data_ptr())
            leaves[g].sync()
        totals = published(gathered, G, R)
        for g in range(G):  # what the leaves publish: their store's running sums (server.go:235-250)
            res = leaves[g].resources(safe=False)
            assert totals[g][0].tobytes() == res["sum_wants"].tobytes()
            assert totals[g][1].tobytes() == res["count"].tobytes()
            assert totals[g][2] == model_flags(totals[g][0], totals[g][1])
        reqs = [M.server_request(*totals[g][:2]) for g in range(G)]
        resp = model.round(now, reqs)
        pre = [leaf_snapshot(leaves[g], tpl[g]) for g in range(G)]
        exchange_all(L, roots, leaves, gathered, G, now)
        for g in range(G):
            if reqs[g] is not None:
                tpl[g] = M.leaf_templates(tpl[g], g, resp, model.cfg)
            assert_root_equal(roots[g], model, f"G={G} round {t} root copy {g}")
            assert_cfg_equal(leaves[g].config(), tpl[g], f"G={G} round {t} leaf {g}")
        for g in range(G):
            leaves[g].apportion(now, writeback=True)
            gets, exp = leaves[g].leases()
            ref = O.apportion(M.with_config(pre[g], tpl[g]), now)
            assert_leases_match(pre[g], gets, exp, ref, f"G={G} round {t} leaf {g}")
            cap, ex, ref_s = leaves[g].leases_proto()
            live = exp != W.RELEASED
            so = pre[g]["seg_off"]
            refresh_row = np.repeat(tpl[g]["refresh_interval_s"], np.diff(so))
            np.testing.assert_array_equal(ref_s[live], refresh_row[live])  # the root's refresh interval
            if clients and t < 3:  # every leaf resource dense after a writeback tick until the
                # last round, where the 20-s default template's followers lapse
                assert leaves[g].store_stats()["dense_resources"] == R, f"G={G} round {t} leaf {g}"
    for e in leaves + roots:
        e.close()


@pytest.mark.parametrize("G", [2, 4, 8, 64])
def test_root_round_grants_stay_within_capacity(G):
    """G servers that each want more than a resource's capacity.  The
    root decides their requests one after another (resource.go:103-104), so on the
    first exchange FairShare grants C, 0, 0, ... and ProportionalShare the same
    (not G x C); later rounds share it out as the sequential model does.  Every
    round: Σ_g grants <= C per resource, the root rows equal the model's bit for
    bit and each leaf template's capacity is its grant."""
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    L = _lib.lib()
    R = 37
    kind = np.where(np.arange(R) % 2 == 0, W.FAIR_SHARE, W.PROPORTIONAL_SHARE).astype(np.int32)
    rcfg = {"kind": kind, "capacity": np.full(R, 100.0), "lease_length_s": np.full(R, 30, np.int64),
            "refresh_interval_s": np.full(R, 5, np.int64), "learning_end_ns": np.full(R, W.INT64_MIN, np.int64),
            "parent_expiry_ns": np.full(R, W.INT64_MAX, np.int64), "safe_capacity": np.full(R, np.nan)}
    roots = [root_engine(rcfg, G)]
    leaf = Engine(0)
    leaf.load(M.with_config(W.uniform(R, 20, kind=W.FAIR_SHARE, seed=1), M.default_config(R)))
    model = M.Root(rcfg, G)
    rng = np.random.default_rng(G)
    gathered = torch.zeros((G * (R + 1), 2), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream, written on the context's
    for t, now in enumerate([NOW, NOW + 5 * W.NS, NOW + 10 * W.NS]):
        sw = rng.uniform(100.0, 300.0, (G, R))  # every server wants more than C
        cnt = rng.integers(1, 40, (G, R)).astype(np.int64)
        gathered.copy_(torch.from_numpy(blocks(sw, cnt)))
        resp = model.round(now, [M.server_request(sw[g], cnt[g]) for g in range(G)])
        _lib.check(L.dm_hier_root_tick(roots[0]._ctx, gathered.data_ptr(), G, now, leaf._ctx, 0), roots[0]._ctx)
        roots[0].sync()
        leaf.sync()
        assert_root_equal(roots[0], model, f"G={G} round {t}")
        grants = np.array([[resp[(g, r)].has for r in range(R)] for g in range(G)])
        assert np.all(grants.sum(axis=0) <= 100.0 * (1 + 1e-12)), (t, grants.sum(axis=0).max())
        if t == 0:
            np.testing.assert_array_equal(grants[0], np.full(R, 100.0))
            assert np.all(grants[1:] == 0.0)
        np.testing.assert_array_equal(leaf.config()["capacity"], grants[0])
    for e in roots + [leaf]:
        e.close()


def test_rejected_server_keeps_its_templates_and_root_rows():
    """server.go:863-866: a band with num_clients < 1 fails the server's whole
    GetServerCapacity (InvalidArgument): that server requests nothing this round,
    its root leases stay, its leaf templates stay (performRequests returns before
    LoadConfig, :268-272); the other servers' round is unaffected.  A Count beyond
    the root's 32-bit column is rejected the same way, never clamped."""
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick
    torch.cuda.set_device(0)
    L = _lib.lib()
    R, G = 16, 3
    rng = np.random.default_rng(5)
    rcfg = root_config(R, rng)
    rcfg["learning_end_ns"][:] = W.INT64_MIN
    model = M.Root(rcfg, G)
    roots = [root_engine(rcfg, G) for _ in range(G)]
    leaves, tpl = [], []
    for g in range(G):
        s = W.uniform(R, 10, kind=W.FAIR_SHARE, seed=40 + g)
        cfg = M.default_config(R)
        e = Engine(0)
        e.load(M.with_config(s, cfg))
        leaves.append(e)
        tpl.append(cfg)
    sw = rng.uniform(10.0, 900.0, (G, R))
    cnt = rng.integers(1, 40, (G, R)).astype(np.int64)
    for t, (bad, value) in enumerate([(None, None), (1, 0), (2, 2**31), (None, None)]):
        c = cnt.copy()
        if bad is not None:
            c[bad, 5] = value
        flags = [model_flags(sw[g], c[g]) for g in range(G)]
        gathered = torch.from_numpy(blocks(sw, c, flags)).to("cuda")
        reqs = [M.server_request(sw[g], c[g]) for g in range(G)]
        assert [r is None for r in reqs] == [f != 0 for f in flags]
        now = NOW + t * W.NS
        resp = model.round(now, reqs)
        exchange_all(L, roots, leaves, gathered, G, now)
        st = np.zeros(G, np.uint32)
        nbad = _lib.check(L.dm_hier_status(roots[0]._ctx, st.ctypes.data, G), roots[0]._ctx)
        want = np.zeros(G, np.uint32)
        if bad is not None:
            want[bad] = _lib.DM_HIER_INVALID if value < 1 else _lib.DM_HIER_COUNT_RANGE
        np.testing.assert_array_equal(st, want)
        assert nbad == int((want != 0).sum())
        for g in range(G):
            if reqs[g] is not None:
                tpl[g] = M.leaf_templates(tpl[g], g, resp, model.cfg)
            assert_root_equal(roots[g], model, f"round {t} root {g}")
            assert_cfg_equal(leaves[g].config(), tpl[g], f"round {t} leaf {g}")
    # HierarchicalTick.check() raises for a rejected server
    ht = HierarchicalTick(torch, leaves[0], roots[0], R, G, 0, lambda src, dst: None)
    c = cnt.copy()
    c[0, 3] = 0
    ht.gathered[0].copy_(torch.from_numpy(blocks(sw, c, [model_flags(sw[g], c[g]) for g in range(G)])))
    L.dm_hier_root_tick(roots[0]._ctx, ht.gathered[0].data_ptr(), G, NOW + 9 * W.NS, leaves[0]._ctx, 0)
    with pytest.raises(_lib.DmError):
        ht.check()
    for e in leaves + roots:
        e.close()


@pytest.mark.parametrize("case", KATS["hierarchy"], ids=lambda c: c["name"])
def test_intermediate_server_update_kat(case):
    """server_test.go:574-658 through the product: an intermediate whose store holds
    a downstream server's band (wants 100, 10 subclients) grants 0 under the "*"
    default template, then 100 once its exchange with the root (FairShare, capacity
    100) has run."""
    import torch
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick
    torch.cuda.set_device(0)
    rt, it, band = case["root"], case["intermediate_default"], case["band"]
    leaf_cfg = {"kind": [it["kind"]], "capacity": [float(it["capacity"])], "lease_length_s": [it["lease_length"]],
                "refresh_interval_s": [it["refresh_interval"]], "learning_end_ns": [W.INT64_MIN],
                "parent_expiry_ns": [W.INT64_MAX], "safe_capacity": [float(it["safe_capacity"])]}
    leaf = Engine(0)
    leaf.load(M.with_config(W.make_snapshot([1], [band["wants"]], [0.0], [band["num_clients"]], [NOW + 60 * W.NS],
                                            W.FAIR_SHARE, 0.0), leaf_cfg))
    leaf.apportion(NOW, writeback=True)
    assert leaf.leases()[0][0] == case["gets_before_exchange"]
    rcfg = {"kind": np.array([rt["kind"]], np.int32), "capacity": np.array([float(rt["capacity"])]),
            "lease_length_s": np.array([rt["lease_length"]]), "refresh_interval_s": np.array([rt["refresh_interval"]]),
            "learning_end_ns": np.array([W.INT64_MIN]), "parent_expiry_ns": np.array([W.INT64_MAX]),
            "safe_capacity": np.array([np.nan])}
    root = root_engine(rcfg, 1)
    ht = HierarchicalTick(torch, leaf, root, 1, 1, 0, lambda src, dst: dst.copy_(src))
    ht.tick(NOW + W.NS)  # the exchange, then the intermediate decides again
    leaf.sync()
    ht.check()
    assert leaf.leases()[0][0] == case["gets_after_exchange"]
    assert leaf.config()["capacity"][0] == case["gets_after_exchange"]
    leaf.close()
    root.close()


def test_hierarchical_tick_shares_one_stream_and_matches_synchronous_steps():
    """HierarchicalTick orders publish -> gather -> root round -> templates -> leaf
    tick on one stream (not torch's null stream, which dm_set_stream cannot
    select): three asynchronous steps leave the same leaf leases as the same steps
    run with a sync after every stage."""
    import torch
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick, root_snapshot
    torch.cuda.set_device(0)
    R = 300
    snap = W.uniform(R, 200, kind=W.FAIR_SHARE, seed=77, capacity=1000.0)

    def gather(src, dst):
        dst.copy_(src)

    outs = []
    for sync_each in (False, True):
        leaf, root = Engine(0), Engine(0)
        leaf.load(snap)
        root.load(root_snapshot(R, 1, W.FAIR_SHARE, np.asarray(snap["capacity"]), lease_length_s=20))
        ht = HierarchicalTick(torch, leaf, root, R, 1, 0, gather)
        assert leaf.stream == root.stream == ht.stream.cuda_stream != 0
        for t in range(3):
            if sync_each:
                ht.exchange(NOW + t * W.NS)
                leaf.sync()
                root.sync()
                leaf.apportion(NOW + t * W.NS, writeback=True)
            else:
                ht.tick(NOW + t * W.NS, asynchronous=True)
        leaf.sync()
        outs.append(leaf.leases())
        leaf.close()
        root.close()
    (g1, e1), (g2, e2) = outs
    assert g1.tobytes() == g2.tobytes() and e1.tobytes() == e2.tobytes()


def test_publish_carries_the_roots_validation():
    """dm_publish_totals: record 1 + r = {SumWants, Count} of resource r; record 0 =
    the flags the root's GetServerCapacity would raise for this request
    (server.go:858-868): a band (SumWants > 0) with Count < 1 -> DM_HIER_INVALID, a
    Count beyond the root's 32-bit column -> DM_HIER_COUNT_RANGE; a resource with
    Count < 1 but no wants is no band and raises nothing."""
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    cases = {
        "ok": ([5, 7, 300], {}),
        "zero_count_no_wants": ([3, 2], {"sub0": 0, "wants0": 0.0}),
        "zero_count_band": ([3, 2, 600], {"sub0": 0}),
        "count_range": ([2, 1000], {"big0": True}),
    }
    for name, (sizes, how) in cases.items():
        sizes = np.asarray(sizes, dtype=np.int64)
        N = int(sizes.sum())
        sub = np.ones(N, np.int64)
        wants = np.full(N, 3.0)
        if "sub0" in how:
            sub[:sizes[0]] = 0
        if "wants0" in how:
            wants[:sizes[0]] = 0.0
        if "big0" in how:
            sub[:2] = 2**31 - 2
        snap = W.make_snapshot(sizes, wants, np.zeros(N), sub, np.full(N, NOW + 60 * W.NS), W.FAIR_SHARE, 100.0)
        R = len(sizes)
        buf = torch.full((R + 3, 2), -7.0, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()  # filled on torch's stream, written on the context's
        with Engine(0) as e:
            e.load(snap)
            for _ in range(2):  # twice: the flag accumulator returns to zero after each launch
                e.publish_totals(buf.data_ptr())
                e.sync()
                rec = buf.cpu().numpy()
                (sw, cnt, flags), = published(buf, 1, R)
                np.testing.assert_array_equal(sw, snap["agg_sum_wants"])
                np.testing.assert_array_equal(cnt, snap["agg_count"])
                assert flags == model_flags(snap["agg_sum_wants"], snap["agg_count"]), name
                assert rec[0, 1] == 0.0 and np.all(rec[R + 1:] == -7.0), name  # nothing past the block
        want = {"ok": 0, "zero_count_no_wants": 0, "zero_count_band": _lib.DM_HIER_INVALID,
                "count_range": _lib.DM_HIER_COUNT_RANGE}[name]
        assert flags == want, (name, flags)


def _shard_rows(model, lo, R):
    """The model's root rows in the sharded device layout: resource r's one row is its
    owner's (server g with lo[g] <= r < lo[g + 1])."""
    G = model.G
    rows = model.rows()
    owner = np.searchsorted(lo, np.arange(R), side="right") - 1
    idx = np.arange(R) * G + owner
    return {k: v[idx] for k, v in rows.items()}


def _shard_templates(prev, g, resp, root_cfg, lo):
    """Server g's templates after an exchange, on its own resources [lo[g], lo[g+1])."""
    a, b = int(lo[g]), int(lo[g + 1])
    local = {(g, r - a): l for (h, r), l in resp.items() if h == g and a <= r < b}
    cfg = {k: np.asarray(root_cfg[k])[a:b] for k in CFG_FIELDS_ALL}
    return M.leaf_templates(prev, g, local, cfg)


CFG_FIELDS_ALL = W.CFG_FIELDS


@pytest.mark.parametrize("pipelined,large", [(False, False), (1, False), (1, True), (2, False)])
def test_sharded_exchange_matches_the_reference_model(pipelined, large):
    """configs[3]'s layout: resources sharded by id over G servers,
    each server an intermediate of its own range; the root (one row per resource,
    its owner's) evaluated redundantly by every server from the gathered blocks.
    Pipelined (dm_hier_pipeline): each leaf tick takes the templates of the exchange
    enqueued before the previous tick (one tick of lag), or (pipelined = 2) one tick
    later still (the lag bench.py uses when the exchange has a stream of its own).  Every step: root copies
    bit for bit against the model, every leaf's templates bit for bit, leaf leases
    against the oracle on the leaf's store under the templates the model says that
    tick used.  `large`: some leaf resources above 4096 rows, so the leaves' ticks run
    the large-resource chain (its steady-state form, without pass B's chunk launch,
    from the second tick) under templates that change kind and capacity."""
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import partition, root_snapshot
    torch.cuda.set_device(0)
    L = _lib.lib()
    G = 3
    rng = np.random.default_rng(31 + pipelined + 2 * large)
    sizes = rng.integers(5, 700, 60)
    if large:
        sizes[rng.choice(60, 6, replace=False)] = rng.integers(4097, 20000, 6)
    R = len(sizes)
    lo = partition(sizes, G)
    S = 1 + int(np.diff(lo).max())
    rcfg = root_config(R, rng)
    full = W.make_snapshot(sizes, rng.uniform(0.2, 3.0, int(sizes.sum())) * 1000.0 / np.repeat(sizes, sizes),
                           0.0, 1, NOW + 60 * W.NS, W.FAIR_SHARE, 1000.0)
    leaves, roots, tpl = [], [], []
    for g in range(G):
        shard = W.subset(full, np.arange(lo[g], lo[g + 1]))
        cfg = M.default_config(int(lo[g + 1] - lo[g]))
        e = Engine(0)
        e.load(M.with_config(shard, cfg))
        if pipelined:
            _lib.check(L.dm_hier_pipeline(e._ctx, int(pipelined)), e._ctx)
        leaves.append(e)
        tpl.append(cfg)
        root = Engine(0)
        root.load(M.with_config(root_snapshot(R, 1, W.FAIR_SHARE, 1.0), rcfg))
        _lib.check(L.dm_hier_layout(root._ctx, G, lo.ctypes.data, S), root._ctx)
        roots.append(root)
    model = M.Root(rcfg, G)
    gathered = torch.zeros((G * S, 2), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream, written on the context's
    staged = []  # templates after each exchange, oldest first (pipelined)
    for t, now in enumerate([NOW, NOW + 5 * W.NS, NOW + 9 * W.NS, NOW + 30 * W.NS, NOW + 31 * W.NS]):
        lag = int(pipelined)
        used = tpl if not pipelined else (staged[t - 1 - lag] if t >= 1 + lag else
                                          [M.default_config(int(lo[g + 1] - lo[g])) for g in range(G)])
        if pipelined:  # tick first (it takes the exchange of two steps ago), then this step's exchange
            for g in range(G):
                pre = leaf_snapshot(leaves[g], used[g])
                leaves[g].apportion(now, writeback=True)
                assert_cfg_equal(leaves[g].config(), used[g], f"step {t} leaf {g} templates in use")
                gets, exp = leaves[g].leases()
                assert_leases_match(pre, gets, exp, O.apportion(pre, now), f"step {t} leaf {g}")
        for g in range(G):
            leaves[g].publish_totals(gathered[g * S:(g + 1) * S].data_ptr())
            leaves[g].sync()
        blocks_ = published(gathered, G, S - 1, S)
        reqs = []
        for g in range(G):
            n = int(lo[g + 1] - lo[g])
            sw, cnt = blocks_[g][0][:n], blocks_[g][1][:n]
            req = M.server_request(sw, cnt)
            reqs.append(None if req is None else {int(lo[g]) + r: v for r, v in req.items()})
        resp = model.round(now, reqs)
        for g in range(G):
            _lib.check(L.dm_hier_root_tick(roots[g]._ctx, gathered.data_ptr(), G, now, leaves[g]._ctx, g), roots[g]._ctx)
        for e in roots + leaves:
            e.sync()
        rows = _shard_rows(model, lo, R)
        sums = model.sums()
        for g in range(G):
            # each rank decides the root round over its own range only (the other ranks
            # decide theirs): root copy g is compared on [lo[g], lo[g+1]), and the rows
            # outside it must still be the loaded (all released) ones
            a, b = int(lo[g]), int(lo[g + 1])
            st, res = roots[g].read_store(), roots[g].resources(safe=False)
            for k in ("has", "wants", "subclients", "expiry_ns"):
                assert st[k][a:b].tobytes() == rows[k][a:b].tobytes(), f"step {t} root copy {g}: {k}"
            assert np.all(st["expiry_ns"][:a] == W.RELEASED) and np.all(st["expiry_ns"][b:] == W.RELEASED), \
                f"step {t} root copy {g} decided resources outside its range"
            for k in ("count", "sum_has", "sum_wants"):
                assert res[k][a:b].tobytes() == sums[k][a:b].tobytes(), f"step {t} root copy {g}: running {k}"
        new = [tpl[g] if reqs[g] is None else _shard_templates(tpl[g], g, resp, model.cfg, lo) for g in range(G)]
        tpl = new
        if pipelined:
            staged.append(new)
        else:
            for g in range(G):
                assert_cfg_equal(leaves[g].config(), tpl[g], f"step {t} leaf {g}")
                pre = leaf_snapshot(leaves[g], tpl[g])
                leaves[g].apportion(now, writeback=True)
                gets, exp = leaves[g].leases()
                assert_leases_match(pre, gets, exp, O.apportion(pre, now), f"step {t} leaf {g}")
        for (g, r), l in resp.items():  # one request per resource: FairShare / PS / Static never exceed C
            if rcfg["kind"][r] != W.NO_ALGORITHM:
                assert l.has <= rcfg["capacity"][r] * (1 + 1e-12), (t, g, r)
    for e in leaves + roots:
        e.close()


def test_publish_ring_matches_publish_totals():
    """dm_publish_ring: writeback tick k writes into ring buffer k % 3 exactly what
    dm_publish_totals writes after it (records bit for bit, validation flags in record
    0 -- here a band with Count 0 from the second tick on), every size bin and kind, and
    clears the next buffer's flags; a non-writeback tick publishes nothing."""
    import ctypes
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    from parity_util import binned_sizes, snapshot_with_sizes
    torch.cuda.set_device(0)
    L = _lib.lib()
    rng = np.random.default_rng(61)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, per_bin=2), hetero=False)
    R = len(snap["seg_off"]) - 1
    ring = [torch.full((R + 1, 2), -1.0, dtype=torch.float64, device="cuda") for _ in range(3)]
    ref = torch.zeros((R + 1, 2), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # the fills run on torch's stream: done before the library writes the buffers
    with Engine(0) as e:
        e.load(snap)
        ptrs = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in ring])
        _lib.check(L.dm_publish_ring(e._ctx, 3, ptrs), e._ctx)
        for k in range(5):
            if k == 1:  # a resource whose rows all carry 0 subclients: Count 0 with SumWants > 0
                so = e.seg_off
                r = int(np.flatnonzero(np.diff(so) > 3)[0])
                rows = np.arange(so[r], so[r + 1])
                e.upsert(rows, np.zeros(len(rows)), np.full(len(rows), 2.0), np.zeros(len(rows), np.int64),
                         np.full(len(rows), NOW + 600 * W.NS))
            e.apportion(NOW + k * W.NS, writeback=True)
            e.publish_totals(ref.data_ptr())
            e.sync()
            got, want = ring[k % 3].cpu().numpy(), ref.cpu().numpy()
            assert got.tobytes() == want.tobytes(), f"tick {k}"
            assert (int(got[0, 0:1].view(np.int64)[0]) != 0) == (k >= 1), f"tick {k} flags"
            assert ring[(k + 1) % 3].cpu().numpy()[0].tobytes() == np.zeros(2).tobytes()  # next flags cleared
        before = [t.cpu().numpy().copy() for t in ring]
        e.apportion(NOW + 9 * W.NS)  # no writeback: no publish
        e.sync()
        for t, b in zip(ring, before):
            assert t.cpu().numpy().tobytes() == b.tobytes()


def test_stream_wait_orders_a_foreign_stream_after_the_tick():
    """dm_stream_wait (stream memory write + wait, not events): a torch stream that
    snapshots the published block right after dm_stream_wait sees the tick's block,
    never the previous one -- ticks forked over the auxiliary streams with deferred
    joins (DM_DEFER_JOIN), wants changed between ticks so every block differs, and a
    store big enough (8M leases) that an unordered copy would overtake the tick."""
    import ctypes
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    L = _lib.lib()
    sizes = np.concatenate([np.full(7000, 1000), np.full(200, 5000), np.full(2000, 40), np.full(1, 50_000)])
    N, R = int(sizes.sum()), len(sizes)
    snap = W.make_snapshot(sizes, np.ones(N), np.zeros(N), 1, np.full(N, NOW + 600 * W.NS), W.FAIR_SHARE, 1e6,
                           300, 5)
    ring = [torch.zeros((R + 1, 2), dtype=torch.float64, device="cuda") for _ in range(3)]
    xs = torch.cuda.Stream()
    torch.cuda.synchronize()  # the fills run on torch's stream
    with Engine(0) as e:
        e.load(snap)
        ptrs = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in ring])
        _lib.check(L.dm_publish_ring(e._ctx, 3, ptrs), e._ctx)
        shots, vals = [], []
        for k in range(6):
            v = 1.0 + k
            e.update_wants(np.arange(N, dtype=np.int64), np.full(N, v))
            e.apportion(NOW + k * W.NS, writeback=True, asynchronous=True, defer_join=True)
            e.stream_wait(xs.cuda_stream)
            with torch.cuda.stream(xs):
                shots.append(ring[k % 3].clone())
            vals.append(v)
        e.sync()
        torch.cuda.synchronize()
    for k, (s, v) in enumerate(zip(shots, vals)):
        got = s.cpu().numpy()[1:, 0]
        assert np.array_equal(got, sizes * v), f"tick {k}: block of another tick"


@pytest.mark.parametrize("G,native", [(1, "local"), (3, "local"), (3, "rccl")])
def test_native_step_matches_the_python_step(G, native):
    """dm_hier_step (the leaf tick and the exchange in one library call, dm_hier_attach)
    against the same pipelined sequence run from Python (HierarchicalTick without
    `native`), with the block gathered in place / copied into its slot ("local") or by
    ncclAllGather over a one-rank communicator of the library's own ("rccl": dlopen'd
    librccl, dm_rccl_unique_id, dm_hier_comm_init): server 0 of G, sharded, the other servers' blocks synthesized from their
    shards' totals (as bench.py --rehearse-shard), its own block copied into its slot
    each step.  Leases, templates in use, root rows and running sums, bit for bit, over
    steps whose templates change; and against the reference model for the root rows."""
    import torch
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick, partition, rccl_unique_id, root_snapshot
    torch.cuda.set_device(0)
    rng = np.random.default_rng(404 + G)
    sizes = rng.integers(5, 900, 40)
    R = len(sizes)
    lo = partition(sizes, G)
    S = 1 + int(np.diff(lo).max())
    rcfg = root_config(R, rng)
    full = W.make_snapshot(sizes, rng.uniform(0.2, 3.0, int(sizes.sum())) * 1000.0 / np.repeat(sizes, sizes),
                           0.0, 1, NOW + 60 * W.NS, W.FAIR_SHARE, 1000.0)
    others = np.zeros((G * S, 2))
    for j in range(1, G):
        sj = W.subset(full, np.arange(lo[j], lo[j + 1]))
        n = int(lo[j + 1] - lo[j])
        others[j * S + 1:j * S + 1 + n, 0] = sj["agg_sum_wants"]
        others[j * S + 1:j * S + 1 + n, 1] = np.asarray(sj["agg_count"], np.int64).view(np.float64)
    shard = W.subset(full, np.arange(lo[0], lo[1]))
    runs = []
    for mode in (native, None):
        leaf, root = Engine(0), Engine(0)
        leaf.load(M.with_config(shard, M.default_config(int(lo[1] - lo[0]))))
        root.load(M.with_config(root_snapshot(R, 1, W.FAIR_SHARE, 1.0), rcfg))

        def gather(src, dst):
            dst[0:S].copy_(src)
        # "rccl": the library's own communicator, here of one rank (server 0's block lands in
        # slot 0 through ncclAllGather): the RCCL leg's plumbing on one GPU
        kw = {"comm_id": rccl_unique_id(), "comm_ranks": 1} if mode == "rccl" else {}
        ht = HierarchicalTick(torch, leaf, root, R, G, 0, gather, shard_lo=lo, pipelined=True, native=mode, **kw)
        if mode == "rccl":  # what RCCL itself counts (dm_hier_comm_info): one rank, this one
            assert ht.comm_info() == (1, 0)
        else:
            assert ht.comm_info() is None
        if G > 1:
            ht.gathered[0].copy_(torch.from_numpy(others).to(ht.gathered[0].device))
        out = []
        for t, now in enumerate([NOW, NOW + 5 * W.NS, NOW + 9 * W.NS, NOW + 14 * W.NS, NOW + 19 * W.NS]):
            ht.tick(now)
            ht.sync()
            out.append((leaf.leases(), leaf.config(), root.read_store(), root.resources(safe=False)))
        runs.append(out)
        leaf.close()
        root.close()
    for t, (a, b) in enumerate(zip(*runs)):
        for x, y in zip(a[0], b[0]):
            assert x.tobytes() == y.tobytes(), f"step {t}: leases"
        assert_cfg_equal(a[1], b[1], f"step {t}: templates")
        for k in ("has", "wants", "subclients", "expiry_ns"):
            assert a[2][k].tobytes() == b[2][k].tobytes(), f"step {t}: root {k}"
        for k in ("count", "sum_has", "sum_wants"):
            assert a[3][k].tobytes() == b[3][k].tobytes(), f"step {t}: root running {k}"


def test_native_step_with_stream_parts_matches_the_python_step():
    """The N = 8 rehearsal's shape with a leaf whose one workgroup bin qualifies for two
    stream parts (dm_plan_info "stream_parts"): the Python sequence (HierarchicalTick
    without `native`, its exchange on a stream of its own) keeps the parts -- ticks in
    two unjoined parts, the root round waiting on both parts' tick events, the template
    slots' reuse likewise -- while dm_hier_attach turns them off (the exchange's waits
    cost more than the parts gain).  dm_hier_step issued back to back with nothing read
    between the steps, and synced after each, against the Python sequence synced after
    each: leases, templates in use, root rows and running sums bit for bit."""
    import torch
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick, partition, root_snapshot
    torch.cuda.set_device(0)
    rng = np.random.default_rng(808)
    G = 3
    sizes = rng.integers(257, 400, G * 4200)
    R = len(sizes)
    lo = partition(sizes, G)
    S = 1 + int(np.diff(lo).max())
    rcfg = root_config(R, rng)
    full = W.make_snapshot(sizes, rng.uniform(0.2, 3.0, int(sizes.sum())) * 1000.0 / np.repeat(sizes, sizes),
                           0.0, 1, NOW + 60 * W.NS, W.FAIR_SHARE, 1000.0)
    others = np.zeros((G * S, 2))
    for j in range(1, G):
        sj = W.subset(full, np.arange(lo[j], lo[j + 1]))
        n = int(lo[j + 1] - lo[j])
        others[j * S + 1:j * S + 1 + n, 0] = sj["agg_sum_wants"]
        others[j * S + 1:j * S + 1 + n, 1] = np.asarray(sj["agg_count"], np.int64).view(np.float64)
    shard = W.subset(full, np.arange(lo[0], lo[1]))
    steps = [NOW + t * W.NS for t in (0, 2, 5, 9, 14, 15, 19, 24, 30, 31)]
    runs = {}
    for mode, sync_each in (("local", False), ("local", True), (None, True)):
        leaf, root = Engine(0), Engine(0)
        leaf.load(M.with_config(shard, M.default_config(int(lo[1] - lo[0]))))
        root.load(M.with_config(root_snapshot(R, 1, W.FAIR_SHARE, 1.0), rcfg))
        assert leaf.plan_info()["stream_parts"] == 2

        def gather(src, dst):
            dst[0:S].copy_(src)
        ht = HierarchicalTick(torch, leaf, root, R, G, 0, gather, shard_lo=lo, pipelined=True, native=mode)
        assert leaf.plan_info()["stream_parts"] == (1 if mode else 2)
        ht.gathered[0].copy_(torch.from_numpy(others).to(ht.gathered[0].device))
        torch.cuda.synchronize()
        out = []
        for now in steps:
            ht.tick(now, asynchronous=not sync_each)
            if sync_each:
                ht.sync()
                out.append((leaf.leases(), leaf.config(), root.read_store(), root.resources(safe=False)))
        ht.sync()
        ht.check()
        out.append((leaf.leases(), leaf.config(), root.read_store(), root.resources(safe=False)))
        runs[(mode, sync_each)] = out
        leaf.close()
        root.close()

    def same(a, b, label):
        for x, y in zip(a[0], b[0]):
            assert x.tobytes() == y.tobytes(), f"{label}: leases"
        assert_cfg_equal(a[1], b[1], f"{label}: templates")
        for k in ("has", "wants", "subclients", "expiry_ns"):
            assert a[2][k].tobytes() == b[2][k].tobytes(), f"{label}: root {k}"
        for k in ("count", "sum_has", "sum_wants"):
            assert a[3][k].tobytes() == b[3][k].tobytes(), f"{label}: root running {k}"
    py = runs[(None, True)]
    for t, (a, b) in enumerate(zip(runs[("local", True)], py)):
        same(a, b, f"synced step {t}")
    same(runs[("local", False)][-1], py[-1], "back-to-back steps, after the last")
