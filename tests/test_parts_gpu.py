"""Stream parts (dm_runtime.cpp plan_parts): a store whose only work class is one
workgroup bin of >= 4096 resources and <= 1 GiB of rows runs that bin as two launches
over its halves, on two auxiliary streams, never joined from tick to tick under
DM_DEFER_JOIN -- so part 0 of tick k + 1 may run beside part 1 of tick k.  The ticks
still are the reference's ticks (store.go:153-181 per resource, resources independent):
  * back-to-back writeback ticks with lapses, a wants refresh between segments (a new
    row epoch: the one-kernel form, then the split form again), against the oracle
    applied tick by tick on a host copy -- every row and every resource's sums;
  * the fused publish (dm_publish_ring) with a Count-0 band in either half: each part
    ORs its flags into its own word of record 0 and clears only that word of the next
    buffer, so the request's flags (the OR of the words) equal dm_publish_totals'.
"""
import ctypes

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import float_close, row_capacity, snapshot_with_sizes

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS


def _host_tick(host, now):
    """The oracle's writeback tick on the host copy (store.go:153-181)."""
    ref = O.apportion(host, now)
    live = ref["expiry_ns"] != W.RELEASED
    host["has"] = np.where(live, ref["gets"], 0.0)
    host["wants"] = np.where(live, host["wants"], 0.0)
    host["subclients"] = np.where(live, host["subclients"], 0)
    host["expiry_ns"] = ref["expiry_ns"].copy()
    W.add_store_sums(host)


def _check(eng, host, label):
    st = eng.read_store()
    np.testing.assert_array_equal(st["expiry_ns"], host["expiry_ns"], err_msg=f"{label}: expiry")
    np.testing.assert_array_equal(st["subclients"], host["subclients"], err_msg=f"{label}: subclients")
    cap = row_capacity(host)
    for k in ("has", "wants"):
        ok = float_close(st[k], host[k], cap)
        assert ok.all(), f"{label}: {int((~ok).sum())} {k} out of tolerance, rows {np.flatnonzero(~ok)[:8].tolist()}"
    res = eng.resources(safe=False)
    np.testing.assert_array_equal(res["count"], host["agg_count"], err_msg=f"{label}: count")
    scale = np.maximum(np.asarray(host["capacity"]), 1.0)
    for k in ("sum_has", "sum_wants"):
        ref = host["agg_" + k]
        assert float_close(res[k], ref, np.maximum(scale, np.abs(ref))).all(), f"{label}: {k}"


@pytest.mark.parametrize("lo,hi,kinds", [(257, 420, (0, 1, 2, 3)), (513, 700, (0, 1, 2, 3)), (513, 1024, (3,))])
def test_parts_back_to_back_ticks_match_the_oracle(lo, hi, kinds):
    """(513-1024 rows, FairShare only: bin 4 on one wave per resource, kBin4Wave)"""
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    rng = np.random.default_rng(lo + len(kinds))
    sizes = rng.integers(lo, hi + 1, 4600)
    snap = snapshot_with_sizes(rng, sizes, kinds=kinds, expired_frac=0.02, learning_frac=0.05)
    W.add_store_sums(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    N = len(snap["wants"])
    with Engine(0) as eng:
        eng.load(snap)
        info = eng.plan_info()
        assert info["stream_parts"] == 2, info
        assert bool(info["bin_shapes"] & 2) == (kinds == (3,)), info  # bin 4's shape
        now = NOW
        for seg in range(3):
            if seg == 2:  # a wants refresh of every seventh row: a new row epoch
                rows = np.arange(5, N, 7, dtype=np.int64)
                vals = rng.uniform(0.1, 4.0, len(rows)) * 10.0
                eng.update_wants(rows, vals)
                live = host["expiry_ns"][rows] != W.RELEASED
                host["wants"][rows[live]] = vals[live]
                W.add_store_sums(host)
            for _ in range(5):  # nothing read between the ticks (bench.py's step)
                now += int(rng.integers(0, 30)) * W.NS
                eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
                _host_tick(host, now)
            eng.sync()
            _check(eng, host, f"segment {seg}")
    print(f"\nparts {lo}-{hi}: {N} leases, 15 ticks against the oracle")


def test_parts_publish_their_own_flags_words():
    import torch
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    L = _lib.lib()
    rng = np.random.default_rng(77)
    R = 4400
    sizes = rng.integers(300, 400, R)
    N = int(sizes.sum())
    snap = W.make_snapshot(sizes, rng.uniform(0.5, 2.0, N), np.zeros(N), 1, np.full(N, NOW + 600 * W.NS),
                           W.FAIR_SHARE, 1000.0)
    so = np.asarray(snap["seg_off"])
    ring = [torch.full((R + 1, 2), -1.0, dtype=torch.float64, device="cuda") for _ in range(3)]
    ref = torch.zeros((R + 1, 2), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # the fills run on torch's stream
    r0, r1 = 17, R - 17  # one resource in each half

    def zero_sub(e, r, v):  # Count 0 with SumWants > 0 (v = 0), or back to one subclient
        rows = np.arange(so[r], so[r + 1])
        e.upsert(rows, np.zeros(len(rows)), np.full(len(rows), 2.0), np.full(len(rows), v, np.int64),
                 np.full(len(rows), NOW + 600 * W.NS))

    with Engine(0) as e:
        e.load(snap)
        assert e.plan_info()["stream_parts"] == 2
        ptrs = (ctypes.c_void_p * 3)(*[t.data_ptr() for t in ring])
        _lib.check(L.dm_publish_ring(e._ctx, 3, ptrs), e._ctx)
        expect = {0: 0, 1: 1, 2: 2, 3: 0, 4: 0, 5: 0, 6: 0}  # which part's word holds the flag
        for k in range(7):
            if k == 1:
                zero_sub(e, r0, 0)
            elif k == 2:
                zero_sub(e, r0, 1)
                zero_sub(e, r1, 0)
            elif k == 3:
                zero_sub(e, r1, 1)
            # ticks 3-6 back to back with nothing between: the split form, parts unjoined
            e.apportion(NOW + k * W.NS, writeback=True, asynchronous=k >= 3, defer_join=k >= 3)
            if k < 3 or k == 6:
                e.publish_totals(ref.data_ptr())
                e.sync()
                got, want = ring[k % 3].cpu().numpy(), ref.cpu().numpy()
                assert got[1:].tobytes() == want[1:].tobytes(), f"tick {k}: records"
                words = got[0:1].view(np.uint32)[0]
                fl = int(words[0]) | int(words[1])
                assert fl == int(want[0:1].view(np.uint32)[0][0]), f"tick {k}: flags {words.tolist()}"
                assert (fl != 0) == (expect[k] != 0), f"tick {k}: flags {words.tolist()}"
                if expect[k]:
                    assert words[expect[k] - 1] != 0 and words[2 - expect[k]] == 0, f"tick {k}: words {words.tolist()}"
                nxt = ring[(k + 1) % 3].cpu().numpy()[0:1].view(np.uint32)[0]
                assert nxt[0] == 0 and nxt[1] == 0, f"tick {k}: next buffer's flags words {nxt.tolist()}"


def test_bin4_shape_follows_the_loaded_kinds():
    """Bin 4 (513-1024 rows) in stream parts takes one wave per resource when most of its
    resources are FairShare (kBin4Wave).  A configuration reload that flips the majority
    after writeback ticks have set dense hints and released-row masks in one shape
    switches the shape (the items go up again without hints); ticks on either side of
    each switch match the oracle.  Without parts the bin keeps 128 x 8."""
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    rng = np.random.default_rng(91)
    sizes = rng.integers(513, 700, 4300)  # >= 4096 items: stream parts
    snap = snapshot_with_sizes(rng, sizes, kinds=(3,), expired_frac=0.03, learning_frac=0.0)
    W.add_store_sums(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    R = len(sizes)
    with Engine(0) as eng:
        eng.load(snap)
        now = NOW
        for step, kind in enumerate([W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.FAIR_SHARE]):
            if step > 0:  # the other kind for every resource: the majority flips
                host["kind"] = np.full(R, kind, np.int32)
                eng.load_config(host)
            info = eng.plan_info()
            assert info["stream_parts"] == 2 and bool(info["bin_shapes"] & 2) == (kind == W.FAIR_SHARE), info
            for _ in range(4):
                now += int(rng.integers(0, 20)) * W.NS
                eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
                _host_tick(host, now)
            eng.sync()
            _check(eng, host, f"kind {kind}")


def test_bin4_without_parts_keeps_its_shape():
    """A FairShare bin 4 that does not run in stream parts (fewer than 4096 items) keeps
    128 x 8 workgroups."""
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    rng = np.random.default_rng(92)
    snap = snapshot_with_sizes(rng, rng.integers(513, 1025, 900), kinds=(3,))
    with Engine(0) as eng:
        eng.load(snap)
        info = eng.plan_info()
        assert info["stream_parts"] == 1 and not info["bin_shapes"] & 2, info


def test_parts_store_turning_general_keeps_its_parts():
    """a store in stream parts (no heterogeneous subclients when it was planned)
    takes an upsert with subclients 3 on some rows of resources in both halves, which
    makes it "maybe general": its FairShare resources with mixed counts go to k_general.
    The parts stay; a tick that may run k_general joins both parts' streams first, so
    back-to-back ticks (nothing read between them) still match the oracle."""
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    rng = np.random.default_rng(99)
    sizes = rng.integers(513, 700, 4600)
    snap = snapshot_with_sizes(rng, sizes, kinds=(2, 3), expired_frac=0.02, learning_frac=0.0)
    hetero = [3, 100, 2400, 4500]
    snap["kind"][hetero] = W.FAIR_SHARE
    snap["parent_expiry_ns"][hetero] = W.INT64_MAX
    W.add_store_sums(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    so = np.asarray(snap["seg_off"])
    with Engine(0) as eng:
        eng.load(snap)
        assert eng.plan_info()["stream_parts"] == 2
        now = NOW
        for _ in range(3):
            eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
            _host_tick(host, now)
        # three subclients on a few live rows of resources in both halves
        rows = np.concatenate([np.arange(so[r], so[r] + 5) for r in hetero])
        rows = rows[host["expiry_ns"][rows] != W.RELEASED]
        exp = np.full(len(rows), now + 600 * W.NS, np.int64)
        eng.upsert(rows, host["has"][rows], host["wants"][rows], np.full(len(rows), 3, np.int64), exp)
        host["subclients"][rows] = 3
        host["expiry_ns"][rows] = exp
        W.add_store_sums(host)
        assert eng.plan_info()["stream_parts"] == 2  # the parts stay
        eng.set_profiling(True)
        for _ in range(4):
            now += int(rng.integers(0, 20)) * W.NS
            eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
            _host_tick(host, now)
        eng.sync()
        _check(eng, host, "after the heterogeneous upsert")
        assert eng.kernel_times().get("general", (0, 0))[0] >= 4  # k_general decided the mixed-count resources
