"""configs[2] sharded over two ranks: the one 1M-resource Zipf
snapshot split by bench.c2_shard_ids (hierarchy.assign_by_class: every rank 1/N of every
size class and the mean predicted tick bytes), one process per rank (gloo; both ranks on GPU 0, the rehearsal of a node),
each rank running bench.py's step -- back-to-back DM_ASYNC | DM_DEFER_JOIN writeback
ticks on its own shard, no collective on the data path (resources are independent,
server.go:810-815; algorithm.go:95-293 has no cross-resource term) -- and checking a
sample of its resources from every size class against the oracle tick by tick
(tests/test_c2_full_gpu.py's sample and host tick).  The ranks then exchange what they
hold over gloo: the shards tile the snapshot exactly, each rank's resources are the ones
bench.c2_shard_ids gives, and the predicted bytes are balanced."""
import os
import socket
import sys

import numpy as np
import pytest

from doorman_amd import workloads as W
from doorman_amd.hierarchy import tick_cost

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from doorman_amd.engine import Engine
        from test_c2_full_gpu import _check, _host_tick, _pick
        snap = bench.make_workload("c2", rank, world, "sharded")
        so = np.asarray(snap["seg_off"])
        rng = np.random.default_rng(70 + rank)
        pick = _pick(snap, rng)
        host = W.subset(snap, pick)
        eng = Engine(0)
        try:
            eng.load(snap)
            eng.set_profiling(True)
            ticks = 0
            for si, seg in enumerate([[W.NOW_NS] * 2, [W.NOW_NS] * 3, [W.NOW_NS + 12 * W.NS] * 2]):
                for now in seg:  # bench.py's step: nothing read between the ticks
                    eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
                    _host_tick(host, now)
                    ticks += 1
                eng.sync()
                _check(eng, host, pick, so, f"rank {rank} segment {si} ({ticks} ticks)")
            kt = {k: v[0] for k, v in eng.kernel_times().items()}
        finally:
            eng.close()
        sizes = np.diff(so)
        mine = {"rank": rank, "resources": len(sizes), "leases": int(sizes.sum()),
                "bytes": float(tick_cost(sizes).sum()), "first_wants": float(snap["wants"][0]),
                "picked": len(pick), "kernels": kt}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        dist.destroy_process_group()
        q.put((rank, "ok", allr))
    except Exception as e:  # noqa: BLE001 (reported to the parent)
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise


def test_c2_sharded_two_ranks_against_the_oracle():
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
        rank, status, allr = q.get(timeout=600)
        assert status == "ok", status
        res[rank] = allr
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allr = res[0]
    assert res[1] == allr  # both ranks saw the same exchange
    sizes = W.zipf_sizes()
    full = W.c2(seed=2)
    seen = np.zeros(len(sizes), np.int32)
    for g, r in enumerate(allr):
        ids = bench.c2_shard_ids(world, g)
        seen[ids] += 1
        assert r["resources"] == len(ids)
        assert r["leases"] == int(sizes[ids].sum())
        assert r["first_wants"] == float(full["wants"][full["seg_off"][ids[0]]])  # the rank's part of ONE snapshot
    assert np.all(seen == 1)  # the shards tile the snapshot
    assert sum(r["leases"] for r in allr) == 13_970_034
    by = [r["bytes"] for r in allr]
    assert max(by) / (sum(by) / world) <= 1.10
    # by class: every rank holds every size class (the speculative chain, the sub-wave groups, the tiles)
    for r in allr:
        assert all(r["kernels"].get(k, 0) >= 3 for k in ("large_spec", "subs_merged", "small_tiles")), r["kernels"]
