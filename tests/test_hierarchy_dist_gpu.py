"""The product hierarchy across processes: two ranks on GPU 0 (gloo, the
rehearsal of the node's RCCL all-gather) each run HierarchicalTick -- publish,
all-gather, their own copy of the root's round, their new templates, their leaf
tick -- for several rounds.  The parent checks every rank against the reference
model (tests/hier_model.py, server.go:227-323 -> :822-901): root copies and
templates bit for bit, leaf leases against the oracle."""
import os
import socket

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
import hier_model as M
from parity_util import assert_leases_match

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS
TIMES = [NOW, NOW + 4 * W.NS, NOW + 30 * W.NS]
R = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _root_cfg():
    rng = np.random.default_rng(11)
    return {"kind": rng.choice([W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.STATIC], R).astype(np.int32),
            "capacity": rng.choice([500.0, 1000.0], R), "lease_length_s": rng.choice([10, 20], R).astype(np.int64),
            "refresh_interval_s": np.full(R, 5, np.int64), "learning_end_ns": np.full(R, W.INT64_MIN, np.int64),
            "parent_expiry_ns": np.full(R, W.INT64_MAX, np.int64),
            "safe_capacity": np.where(np.arange(R) % 3 == 0, 4.5, np.nan)}


def _leaf_snap(rank):
    s = W.uniform(R, 30 + 17 * rank, kind=W.FAIR_SHARE, seed=300 + rank, capacity=1000.0)
    return M.with_config(s, M.default_config(R))


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick
    cfg = _root_cfg()
    N = R * world
    leaf, root = Engine(0), Engine(0)
    leaf.load(_leaf_snap(rank))
    root.load(W.make_snapshot(np.full(R, world), np.zeros(N), np.zeros(N), np.zeros(N, np.int64),
                              np.full(N, W.RELEASED), cfg["kind"], cfg["capacity"], cfg["lease_length_s"],
                              cfg["refresh_interval_s"], cfg["learning_end_ns"], cfg["parent_expiry_ns"],
                              cfg["safe_capacity"]))

    def gather(src, dst):  # through host memory: every rank shares one GPU here
        parts = [torch.empty_like(src, device="cpu") for _ in range(world)]
        dist.all_gather(parts, src.cpu())
        dst.copy_(torch.cat(parts).to(dst.device))

    ht = HierarchicalTick(torch, leaf, root, R, world, rank, gather)
    out = []
    for now in TIMES:
        pre = {**leaf.read_store(), **leaf.resources(safe=False)}
        ht.tick(now)
        leaf.sync()
        ht.check()
        out.append({"pre": pre, "root": {**root.read_store(), **root.resources(safe=False)}, "cfg": leaf.config(),
                    "leases": leaf.leases()})
    q.put((rank, out))
    leaf.close()
    root.close()
    dist.destroy_process_group()


def test_hierarchical_tick_two_processes_matches_the_reference_model():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, out = q.get(timeout=240)
        res[rank] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    model = M.Root(_root_cfg(), world)
    tpl = [M.default_config(R) for _ in range(world)]
    seg_off = [_leaf_snap(g)["seg_off"] for g in range(world)]
    for t, now in enumerate(TIMES):
        reqs = [M.server_request(res[g][t]["pre"]["sum_wants"], res[g][t]["pre"]["count"]) for g in range(world)]
        resp = model.round(now, reqs)
        rows, sums = model.rows(), model.sums()
        for g in range(world):
            got = res[g][t]
            for k in ("has", "wants", "subclients", "expiry_ns"):
                assert got["root"][k].tobytes() == rows[k].tobytes(), (t, g, k)
            for k in ("count", "sum_has", "sum_wants"):
                assert got["root"][k].tobytes() == sums[k].tobytes(), (t, g, k)
            tpl[g] = M.leaf_templates(tpl[g], g, resp, model.cfg)
            for k in W.CFG_FIELDS:
                np.testing.assert_array_equal(got["cfg"][k], tpl[g][k], err_msg=f"round {t} rank {g} {k}")
            pre = got["pre"]
            snap = M.with_config({"seg_off": seg_off[g], "wants": pre["wants"], "has": pre["has"],
                                  "subclients": pre["subclients"], "expiry_ns": pre["expiry_ns"],
                                  "agg_count": pre["count"], "agg_sum_has": pre["sum_has"],
                                  "agg_sum_wants": pre["sum_wants"]}, tpl[g])
            gets, exp = got["leases"]
            assert_leases_match(snap, gets, exp, O.apportion(snap, now), f"round {t} rank {g}")


# ---- configs[3]'s layout: one snapshot sharded by resource id, pipelined exchange ----
RS = 50
SIZES = np.random.default_rng(21).integers(5, 400, RS)
STEPS = [NOW, NOW + 4 * W.NS, NOW + 8 * W.NS, NOW + 30 * W.NS, NOW + 34 * W.NS]


def _full_snap():
    s = W.make_snapshot(SIZES, np.random.default_rng(22).uniform(0.2, 3.0, int(SIZES.sum())) * 1000.0 /
                        np.repeat(SIZES, SIZES), 0.0, 1, NOW + 60 * W.NS, W.FAIR_SHARE, 1000.0)
    return s


def _rank_sharded(rank, world, port, q, lag):
    import traceback
    try:
        _rank_sharded_body(rank, world, port, q, lag)
    except Exception:  # report to the parent instead of leaving it waiting
        q.put((rank, "error: " + traceback.format_exc()))
        raise


def _rank_sharded_body(rank, world, port, q, lag):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from doorman_amd.engine import Engine
    from doorman_amd.hierarchy import HierarchicalTick, partition, root_snapshot
    lo = partition(SIZES, world)
    leaf, root = Engine(0), Engine(0)
    shard = W.subset(_full_snap(), np.arange(lo[rank], lo[rank + 1]))
    leaf.load(M.with_config(shard, M.default_config(int(lo[rank + 1] - lo[rank]))))
    root.load(M.with_config(root_snapshot(RS, 1, W.FAIR_SHARE, 1.0), _root_cfg_s()))

    def gather(src, dst):  # through host memory: every rank shares one GPU here
        parts = [torch.empty_like(src, device="cpu") for _ in range(world)]
        dist.all_gather(parts, src.cpu())
        dst.copy_(torch.cat(parts).to(dst.device))

    ht = HierarchicalTick(torch, leaf, root, RS, world, rank, gather, shard_lo=lo, pipelined=True, lag=lag)
    assert ht.stream.cuda_stream != ht.xstream.cuda_stream
    out = []
    for now in STEPS:
        pre = {**leaf.read_store(), **leaf.resources(safe=False)}
        ht.tick(now)  # the leaf tick (templates of the exchange two steps back), then this step's exchange
        out.append({"pre": pre, "post": leaf.resources(safe=False), "cfg": leaf.config(), "leases": leaf.leases(),
                    "root": {**root.read_store(), **root.resources(safe=False)}, "status": ht.status()})
    q.put((rank, out))
    leaf.close()
    root.close()
    dist.destroy_process_group()


def _root_cfg_s():
    rng = np.random.default_rng(12)
    return {"kind": rng.choice([W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.STATIC], RS).astype(np.int32),
            "capacity": rng.choice([300.0, 1000.0], RS), "lease_length_s": rng.choice([10, 20], RS).astype(np.int64),
            "refresh_interval_s": np.full(RS, 5, np.int64), "learning_end_ns": np.full(RS, W.INT64_MIN, np.int64),
            "parent_expiry_ns": np.full(RS, W.INT64_MAX, np.int64),
            "safe_capacity": np.where(np.arange(RS) % 3 == 0, 4.5, np.nan)}


@pytest.mark.parametrize("lag", [1, 2])
def test_sharded_pipelined_hierarchical_tick_two_processes(lag):
    """bench.py's configs[3] path across processes: the resources of one snapshot
    sharded by id over two ranks, each an intermediate server of its range; every
    step a leaf tick, then the pipelined exchange (publish, all-gather, the root's
    round over each rank's own resources, staged templates taken by the leaf tick
    two steps later).  Root copies bit for bit against the model on both ranks' ranges,
    templates bit for bit, leaf leases against the oracle under the templates the
    model says each tick used."""
    import torch.multiprocessing as mp
    from doorman_amd.hierarchy import partition
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_sharded, args=(r, world, port, q, lag)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, out = q.get(timeout=150)
        assert not isinstance(out, str), out
        res[rank] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lo = partition(SIZES, world)
    rcfg = _root_cfg_s()
    model = M.Root(rcfg, world)
    full = _full_snap()
    seg_off = [W.subset(full, np.arange(lo[g], lo[g + 1]))["seg_off"] for g in range(world)]
    tpl = [M.default_config(int(lo[g + 1] - lo[g])) for g in range(world)]
    staged = []
    owner = np.searchsorted(lo, np.arange(RS), side="right") - 1
    for t, now in enumerate(STEPS):
        used = (staged[t - 1 - lag] if t >= 1 + lag else
                [M.default_config(int(lo[g + 1] - lo[g])) for g in range(world)])
        reqs = []
        for g in range(world):
            got = res[g][t]
            for k in W.CFG_FIELDS:
                np.testing.assert_array_equal(got["cfg"][k], used[g][k], err_msg=f"step {t} rank {g} {k}")
            pre = got["pre"]
            snap = M.with_config({"seg_off": seg_off[g], "wants": pre["wants"], "has": pre["has"],
                                  "subclients": pre["subclients"], "expiry_ns": pre["expiry_ns"],
                                  "agg_count": pre["count"], "agg_sum_has": pre["sum_has"],
                                  "agg_sum_wants": pre["sum_wants"]}, used[g])
            gets, exp = got["leases"]
            assert_leases_match(snap, gets, exp, O.apportion(snap, now), f"step {t} rank {g}")
            req = M.server_request(got["post"]["sum_wants"], got["post"]["count"])
            reqs.append(None if req is None else {int(lo[g]) + r: v for r, v in req.items()})
        for g in range(world):  # every root copy rejects the same servers (a band with Count < 1: the
            # float residual SumWants > 0 of a range whose leases all lapsed, server.go:863-866)
            np.testing.assert_array_equal(res[g][t]["status"] != 0, [r is None for r in reqs])
        resp = model.round(now, reqs)
        rows, sums = model.rows(), model.sums()
        idx = np.arange(RS) * world + owner
        for g in range(world):  # each rank decides the root round over its own range only
            got = res[g][t]["root"]
            a, b = int(lo[g]), int(lo[g + 1])
            for k in ("has", "wants", "subclients", "expiry_ns"):
                assert got[k][a:b].tobytes() == rows[k][idx][a:b].tobytes(), (t, g, k)
            for k in ("count", "sum_has", "sum_wants"):
                assert got[k][a:b].tobytes() == sums[k][a:b].tobytes(), (t, g, k)
        new = []
        for g in range(world):
            a, b = int(lo[g]), int(lo[g + 1])
            local = {(g, r - a): l for (h, r), l in resp.items() if h == g}
            cfg = {k: np.asarray(model.cfg[k])[a:b] for k in W.CFG_FIELDS}
            new.append(tpl[g] if reqs[g] is None else M.leaf_templates(tpl[g], g, local, cfg))
        tpl = new
        staged.append(new)
