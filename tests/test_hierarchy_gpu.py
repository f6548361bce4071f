"""The intermediate-server hierarchy on one GPU: G simulated servers publish
their totals, the gathered records feed the root store (dm_hier_load_root), the
root apportions its G server rows per resource, every server takes its grant
(dm_hier_take_grants) and runs its leaf tick -- all checked against the oracle
model of GetServerCapacity (tests/hier_model.py)."""
import numpy as np
import pytest

from doorman_amd import hierarchy as H
from doorman_amd import workloads as W
from oracle import oracle as O
import hier_model as M
from parity_util import assert_leases_match

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS


@pytest.mark.parametrize("G", [2, 3, 8, 20])
def test_hierarchy_round(G):
    import torch
    from doorman_amd.engine import Engine
    R = 64
    torch.cuda.set_device(0)
    rng = np.random.default_rng(G)
    leaves, snaps = [], []
    for g in range(G):
        s = W.uniform(R, int(rng.integers(5, 300)), kind=W.FAIR_SHARE, seed=10 * G + g, capacity=1000.0)
        s["wants"] *= rng.uniform(0.2, 3.0)  # servers differ in appetite
        if g == 1:
            s["wants"][: len(s["wants"]) // 4] = 0.0  # some resources not requested by server 1
        W.add_store_sums(s)
        e = Engine(0)
        e.load(s)
        leaves.append(e)
        snaps.append(s)
    root = Engine(0)
    rsnap = H.root_snapshot(R, G, W.FAIR_SHARE, 1000.0, lease_length_s=20)
    root.load(rsnap)
    dev = torch.device("cuda", 0)
    gathered = torch.empty((G * R, 2), dtype=torch.float64, device=dev)
    for g, e in enumerate(leaves):
        e.publish_totals(gathered[g * R:(g + 1) * R].data_ptr())
        e.sync()
    from doorman_amd import _lib
    _lib.check(_lib.lib().dm_hier_load_root(root._ctx, gathered.data_ptr(), G, NOW), root._ctx)
    root.apportion(NOW, writeback=True, recompute=True)
    rg, rexp = root.leases()
    # model: totals as published (store SumWants / Count, server.go:241-249)
    host = gathered.cpu().numpy()
    totals = [(host[g * R:(g + 1) * R, 0].copy(), host[g * R:(g + 1) * R, 1].copy().view(np.int64))
              for g in range(G)]
    for g in range(G):
        np.testing.assert_array_equal(totals[g][1], snaps[g]["agg_count"])
    msnap = M.root_from_totals(totals, 1000.0, W.FAIR_SHARE, 20, np.zeros(R * G), NOW)
    mout = O.apportion(msnap, NOW)
    assert_leases_match(msnap, rg, rexp, mout, f"root G={G}")
    for g, e in enumerate(leaves):
        _lib.check(_lib.lib().dm_hier_take_grants(root._ctx, e._ctx, g), root._ctx)
        cap, parent, live = M.grants(msnap, mout, G, g)
        leaf = dict(snaps[g])
        leaf["capacity"] = np.where(live, cap, snaps[g]["capacity"])
        leaf["parent_expiry_ns"] = np.where(live, parent, snaps[g]["parent_expiry_ns"])
        e.apportion(NOW, writeback=False)
        gets, exp = e.leases()
        assert_leases_match(leaf, gets, exp, O.apportion(leaf, NOW), f"leaf {g} of {G}")
        # and past the grant's expiry the leaf's capacity is 0 (resource.go:62-70)
        later = NOW + 25 * W.NS
        e.apportion(later, writeback=False)
        gets2, exp2 = e.leases()
        assert_leases_match(leaf, gets2, exp2, O.apportion(leaf, later), f"leaf {g} after parent expiry")
    for e in leaves + [root]:
        e.close()


def test_hierarchical_tick_shares_one_stream_and_matches_synchronous_steps():
    """HierarchicalTick orders publish -> gather -> root -> grants -> leaf tick on one
    stream (not torch's null stream, which dm_set_stream cannot select): three
    asynchronous steps leave the same leaf leases as the same steps run with a sync
    after every stage."""
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    R = 300
    snap = W.uniform(R, 200, kind=W.FAIR_SHARE, seed=77, capacity=1000.0)

    def gather(src, dst):
        dst.copy_(src)

    outs = []
    for sync_each in (False, True):
        leaf, root = Engine(0), Engine(0)
        leaf.load(snap)
        root.load(H.root_snapshot(R, 1, W.FAIR_SHARE, np.asarray(snap["capacity"]), lease_length_s=20))
        ht = H.HierarchicalTick(torch, leaf, root, R, 1, 0, gather)
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


@pytest.mark.parametrize("G", [1, 2, 3, 8, 20])
def test_hier_root_tick_matches_separate_calls(G):
    """dm_hier_root_tick (one fused launch for G <= 8, the three calls above) leaves
    the root store, its running sums and the leaf's template exactly as
    dm_hier_load_root + dm_apportion(WRITEBACK | AGG_RECOMPUTE) + dm_hier_take_grants;
    two rounds, so the second sees the first's root leases."""
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    R = 257
    rng = np.random.default_rng(100 + G)
    snap = W.uniform(R, 40, kind=W.FAIR_SHARE, seed=5 + G, capacity=1000.0)
    rec = np.empty((G * R, 2))
    rec[:, 0] = rng.uniform(0.0, 600.0, G * R) * (rng.random(G * R) > 0.1)
    rec[:, 1] = rng.integers(0, 50, G * R).astype(np.int64).view(np.float64)
    gathered = torch.from_numpy(rec).to("cuda")
    L = _lib.lib()
    outs = []
    for fused in (True, False):
        leaf, root = Engine(0), Engine(0)
        leaf.load(snap)
        root.load(H.root_snapshot(R, G, W.FAIR_SHARE, np.asarray(snap["capacity"]) * G, lease_length_s=20))
        for t in range(2):
            now = NOW + t * W.NS
            server = (t + G - 1) % G
            if fused:
                _lib.check(L.dm_hier_root_tick(root._ctx, gathered.data_ptr(), G, now, leaf._ctx, server), root._ctx)
            else:
                _lib.check(L.dm_hier_load_root(root._ctx, gathered.data_ptr(), G, now), root._ctx)
                root.apportion(now, writeback=True, recompute=True)
                _lib.check(L.dm_hier_take_grants(root._ctx, leaf._ctx, server), root._ctx)
        root.sync()
        leaf.apportion(NOW + W.NS, writeback=False)
        outs.append((root.read_store(), root.resources(safe=False), leaf.leases()))
        leaf.close()
        root.close()
    (s1, r1, l1), (s2, r2, l2) = outs
    for k in ("has", "wants", "subclients", "expiry_ns"):
        assert s1[k].tobytes() == s2[k].tobytes(), k
    for k in ("count", "sum_has", "sum_wants"):
        assert r1[k].tobytes() == r2[k].tobytes(), k
    assert l1[0].tobytes() == l2[0].tobytes() and l1[1].tobytes() == l2[1].tobytes()
