"""The benched configuration itself under the oracle, at full size.

bench.py's default line is configs[3] at N = 1: rank 0's shard of the one 100M-lease
snapshot (100k resources x 1000 clients, FairShare), the intermediate-server
exchange every step, pipelined beside the next leaf tick (dm_hier_pipeline: each
leaf tick takes the templates of the exchange enqueued two steps before).  This test
builds exactly that (bench.make_workload, bench.c3_bounds, the same root store, the
product HierarchicalTick) and runs six steps, so that from the third tick on the
leaf runs the dense split (k_block_dense<128, 8> + k_block_rest) under templates
that change (the loaded configuration for two ticks, then the root's grants: capacity,
parent expiry, lease length).  Each step:
  * 64 sampled resources (the first, the last and 62 random ones) are decided by the
    oracle (O.apportion) on a host copy of their rows and running sums as they stood
    before the tick, under the templates the hierarchy model (tests/hier_model.py,
    restated from server.go:227-323,822-901) says that tick used; leases must match
    (SURVEY.md §8c bar);
  * every resource's templates in use equal the model's bit for bit;
  * the root rows and running sums of the whole range equal the model's bit for bit;
  * Count == live rows and sumHas == the sum of the live gets over all 100k
    resources (the size-independent properties of a writeback tick), on the last step.
"""
import os
import sys

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
import hier_model as M
from parity_util import assert_leases_match, float_close

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def _sample_snapshot(leaf, cfg, res_ids, so):
    """The sampled resources' rows and running sums as the device holds them now,
    under `cfg` (per-resource columns over the whole leaf), as one oracle snapshot."""
    parts = {k: [] for k in ("wants", "has", "subclients", "expiry_ns")}
    sizes, sums = [], {"count": [], "sum_has": [], "sum_wants": []}
    for r in res_ids:
        a, b = int(so[r]), int(so[r + 1])
        st = leaf.read_store(a, b - a)
        for k in parts:
            parts[k].append(st[k])
        rr = leaf.resources(int(r), 1, safe=False)
        for k in sums:
            sums[k].append(rr[k][0])
        sizes.append(b - a)
    sub = {k: np.asarray(cfg[k])[res_ids] for k in W.CFG_FIELDS}
    snap = W.make_snapshot(np.asarray(sizes), np.concatenate(parts["wants"]), np.concatenate(parts["has"]),
                           np.concatenate(parts["subclients"]), np.concatenate(parts["expiry_ns"]), sub["kind"],
                           sub["capacity"], sub["lease_length_s"], sub["refresh_interval_s"], sub["learning_end_ns"],
                           sub["parent_expiry_ns"], sub["safe_capacity"], aggregates=False)
    snap["agg_count"] = np.asarray(sums["count"], np.int64)
    snap["agg_sum_has"] = np.asarray(sums["sum_has"])
    snap["agg_sum_wants"] = np.asarray(sums["sum_wants"])
    return snap


def test_benched_c3_configuration_against_the_oracle_at_full_size():
    import torch
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick, root_snapshot
    torch.cuda.set_device(0)
    snap = bench.make_workload("c3", 0, 1, "sharded")
    R, N = len(snap["seg_off"]) - 1, len(snap["wants"])
    assert (R, N) == (bench.C3_R, bench.C3_R * bench.C3_CLIENTS)
    so = np.asarray(snap["seg_off"])
    init_cfg = {k: np.broadcast_to(np.asarray(snap[k]), (R,)).copy() for k in W.CFG_FIELDS}
    root_snap = root_snapshot(bench.C3_R, 1, W.FAIR_SHARE, 1000.0, lease_length_s=20)
    root_cfg = {k: np.broadcast_to(np.asarray(root_snap[k]), (R,)).copy() for k in W.CFG_FIELDS}
    leaf, root = Engine(0), Engine(0)
    try:
        leaf.load(snap)
        root.load(root_snap)
        del snap  # 3 GB of host columns: the device holds the store now
        bounds = bench.c3_bounds(1)
        ht = HierarchicalTick(torch, leaf, root, bench.C3_R, 1, 0, None, shard_lo=bounds, pipelined=True)
        model = M.Root(root_cfg, 1)
        rng = np.random.default_rng(2024)
        pick = np.unique(np.concatenate([[0, R - 1], rng.choice(R, 62, replace=False)]))
        leaf.set_profiling(True)  # per-class launch counts: which form each tick ran
        staged = []
        tpl = init_cfg
        now = W.NOW_NS  # bench.py ticks at one instant: nothing lapses, every resource turns dense
        for t in range(6):
            used = staged[t - 2] if t >= 2 else init_cfg
            pre = _sample_snapshot(leaf, used, pick, so)
            ht.tick(now)  # the leaf tick (templates of two exchanges back), then this step's exchange
            ht.sync()
            cfg_now = leaf.config()
            for k in W.CFG_FIELDS:
                a, b = np.asarray(cfg_now[k]), np.asarray(used[k])
                same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
                assert same.all(), f"step {t}: template {k} in use differs at {np.flatnonzero(~same)[:8].tolist()}"
            got = _sample_snapshot(leaf, used, pick, so)
            gets = got["has"]  # a writeback tick writes each lease into the store's has column
            exp = got["expiry_ns"]
            ref = O.apportion(pre, now)
            assert_leases_match(pre, gets, exp, ref, f"step {t}: sampled resources")
            np.testing.assert_array_equal(got["agg_count"], ref["res_count"], err_msg=f"step {t}: count")
            # the exchange this step enqueued: the model's root round on the leaf's totals
            res = leaf.resources(safe=False)
            req = M.server_request(res["sum_wants"], res["count"])
            resp = model.round(now, [req])
            tpl = tpl if req is None else M.leaf_templates(tpl, 0, resp, model.cfg)
            staged.append(tpl)
            st, rres = root.read_store(), root.resources(safe=False)
            rows, sums = model.rows(), model.sums()
            for k in ("has", "wants", "subclients", "expiry_ns"):
                assert st[k].tobytes() == rows[k].tobytes(), f"step {t}: root {k}"
            for k in ("count", "sum_has", "sum_wants"):
                assert rres[k].tobytes() == sums[k].tobytes(), f"step {t}: root running {k}"
        # the dense split ran under the changing templates (every tick from the third on)
        kt = leaf.kernel_times()
        assert kt.get("block128x8_dense", (0, 0))[0] >= 4, kt
        assert leaf.store_stats()["dense_resources"] == R
        # Count == live rows (one subclient each) and sumHas == sum of live gets, every resource
        gets, exp = leaf.leases()
        live = exp != W.RELEASED
        cnt = np.add.reduceat(live.astype(np.int64), so[:-1])
        sh = np.add.reduceat(np.where(live, gets, 0.0), so[:-1])
        res = leaf.resources(safe=False)
        np.testing.assert_array_equal(res["count"], cnt)
        assert float_close(res["sum_has"], sh, np.maximum(np.asarray(tpl["capacity"]), 1.0)).all()
        print(f"\nC3 full size: 6 steps, {len(pick)} sampled resources per step against the oracle, "
              f"templates and root rows bit for bit, Count/sumHas over {R} resources")
    finally:
        leaf.close()
        root.close()
