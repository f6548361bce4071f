"""configs[2]'s benched steady state under the oracle, at full size.

bench.py times configs[2] (C2: 1M resources, Zipf 1..1M clients = 13,970,034 leases,
mixed kinds, 5 % learning) as writeback ticks issued back to back with DM_ASYNC |
DM_DEFER_JOIN, nothing read in between.  That steady state engages paths a first tick
never reaches: the speculative chain (k_large_spec) and its redo by teams (light and
full builds), the sub-wave kernel's pass-A skip, the dense workgroup kernels with
released-row masks and no rest kernel, the alternate gets column.  This test runs
exactly those ticks on bench.make_workload("c2") and, after every synchronised
segment, compares a sample of resources from every size class with the oracle
(O.apportion) applied tick by tick on a host copy of their rows:
  * the 10 largest resources, both sides of every bin and sub-wave shape edge
    (4/5, 6/7, 8/9, 12/13 ... 4096/4097),
    learning, Static and NoAlgorithm resources, and random resources of every class;
  * segment 0 from the load (the first tick takes the four-launch chain: loaded rows
    carry explicit expiries, 1 % of them already past), segment 1 the steady state;
  * between segments 1 and 2 one dm_store_apply (a wants refresh of every tenth row,
    departures, arrivals onto freed rows -- half of them with an expiry that lapses
    before segment 2), so segment 2's first tick has Clean release rows on resources
    of every class (their speculation fails: the redo runs) and segment 3 runs past
    the learning resources' end of learning mode.
Leases (gets bit-exact for the packed class, within SURVEY.md §8c's 1e-9 bar
otherwise), expiries, subclients and counts bit-exact, running sums within the bar.
"""
import os
import sys

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import float_close, row_capacity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def _pick(snap, rng):
    sizes = np.diff(snap["seg_off"])
    R = len(sizes)
    pick = list(range(10))  # the largest (sizes fall with the Zipf rank)
    for e in (4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 512, 1024, 2048, 4096):  # every bin and shape edge
        above = np.flatnonzero(sizes > e)
        below = np.flatnonzero(sizes <= e)
        if len(above):
            pick.append(int(above[-1]))
        if len(below):
            pick.append(int(below[0]))
    classes = [(1, 1), (2, 4), (5, 16), (17, 256), (257, 4096), (4097, 1 << 40)]
    learning = snap["learning_end_ns"] != W.INT64_MIN
    for lo, hi in classes:
        ids = np.flatnonzero((sizes >= lo) & (sizes <= hi))
        pick += rng.choice(ids, min(len(ids), 40), replace=False).tolist()
        for cond in (learning[ids], snap["kind"][ids] == W.STATIC, snap["kind"][ids] == W.NO_ALGORITHM):
            sel = ids[cond]
            if len(sel):
                pick += rng.choice(sel, min(len(sel), 3), replace=False).tolist()
    pick = np.unique(np.asarray(pick, np.int64))
    assert pick[-1] < R
    return pick


def _host_tick(host, now):
    """The oracle's writeback tick on the host copy (store.go:153-181)."""
    ref = O.apportion(host, now)
    live = ref["expiry_ns"] != W.RELEASED
    host["has"] = np.where(live, ref["gets"], 0.0)
    host["wants"] = np.where(live, host["wants"], 0.0)
    host["subclients"] = np.where(live, host["subclients"], 0)
    host["expiry_ns"] = ref["expiry_ns"].copy()
    W.add_store_sums(host)


def _check(eng, host, pick, so, label):
    """Device rows and sums of the picked resources against the host's chained oracle
    ticks; afterwards the host continues from the device's state (rebase), so every
    segment is compared from one shared starting state.

    Sums: the device's running sums must agree with its own rows (self-consistency,
    1e-9 of the magnitudes summed), and with the host's up to what the rows' own
    differences explain.  A fully allocated FairShare resource's grants depend on
    capacity - SumHas (algorithm.go:120: cancellation), so the last ulps of the previous
    tick's SumHas -- tree-ordered on the device, row-ordered on the host, map-ordered in
    Go -- move every avail-bound grant by ~1e-9 relative on the next tick: within the
    per-lease bar, but a direct sum comparison at 1e-9 of the capacity then fails on a
    500k-row resource on alternate ticks."""
    parts = {k: [] for k in ("has", "subclients", "expiry_ns", "wants")}
    for r in pick:
        st = eng.read_store(int(so[r]), int(so[r + 1] - so[r]))
        for k in parts:
            parts[k].append(st[k])
    got = {k: np.concatenate(v) for k, v in parts.items()}
    np.testing.assert_array_equal(got["expiry_ns"], host["expiry_ns"], err_msg=f"{label}: expiry")
    np.testing.assert_array_equal(got["subclients"], host["subclients"], err_msg=f"{label}: subclients")
    cap = row_capacity(host)
    for k in ("has", "wants"):
        ok = float_close(got[k], host[k], cap)
        if not ok.all():
            bad = np.flatnonzero(~ok)[:8]
            raise AssertionError(f"{label}: {int((~ok).sum())} {k} out of tolerance, rows {bad.tolist()}: "
                                 f"{got[k][bad].tolist()} vs {host[k][bad].tolist()}")
    res = [eng.resources(int(r), 1, safe=False) for r in pick]
    cnt = np.asarray([x["count"][0] for x in res])
    np.testing.assert_array_equal(cnt, host["agg_count"], err_msg=f"{label}: count")
    hso = host["seg_off"]
    scale = np.maximum(np.asarray(host["capacity"]), 1.0)
    sizes = np.diff(so)
    dev_sums = {}
    for k in ("has", "wants"):
        v = np.asarray([x["sum_" + k][0] for x in res])
        dev_sums[k] = v
        ref = host["agg_sum_" + k]
        rows_dev = W.segment_sums(got[k], hso)
        rows_host = W.segment_sums(host[k], hso)
        mag = np.maximum(scale, W.segment_sums(np.abs(got[k]), hso))
        self_ok = float_close(v, rows_dev, mag)
        expl = np.abs(v - ref) <= np.abs(rows_dev - rows_host) + 1e-9 * np.maximum(mag, np.abs(ref))
        ok = self_ok & (float_close(v, ref, np.maximum(scale, np.abs(ref))) | expl)
        if not ok.all():
            bad = np.flatnonzero(~ok)[:6]
            raise AssertionError(f"{label}: sum_{k} of {int((~ok).sum())} resources out of tolerance: "
                                 + "; ".join(f"r{int(pick[i])} n={int(sizes[pick[i]])} kind={int(host['kind'][i])} "
                                             f"got {v[i]!r} ref {ref[i]!r} own rows {rows_dev[i]!r} host rows "
                                             f"{rows_host[i]!r} cap {host['capacity'][i]!r}" for i in bad))
    for k in ("has", "wants"):  # rebase: the next segment starts from the device's state
        host[k] = got[k].copy()
        host["agg_sum_" + k] = dev_sums[k].copy()


def test_benched_c2_steady_state_against_the_oracle_at_full_size():
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    snap = bench.make_workload("c2", 0)
    so = np.asarray(snap["seg_off"])
    N = len(snap["wants"])
    assert N == 13_970_034
    rng = np.random.default_rng(2025)
    pick = _pick(snap, rng)
    host = W.subset(snap, pick)
    grow = np.concatenate([np.arange(so[r], so[r + 1]) for r in pick])  # device row of every host row
    eng = Engine(0)
    try:
        eng.load(snap)
        eng.set_profiling(True)
        now0 = W.NOW_NS
        segments = [[now0] * 3, [now0] * 4, [now0 + 5 * W.NS] * 3, [now0 + 12 * W.NS] * 3]
        ticks = 0
        for si, seg in enumerate(segments):
            if si == 2:
                # one round of store updates (bench's configs[4] step shape): a wants refresh of
                # every tenth row (live rows only: a refresh of a released row changes nothing),
                # departures of every hundredth row, arrivals onto every other departed row,
                # half of them with an expiry that has passed by segment 2's ticks
                upd = np.arange(3, N, 10, dtype=np.int64)
                wv = rng.uniform(0.1, 3.0, len(upd)) * 50.0
                gone = np.arange(7, N, 100, dtype=np.int64)
                new = gone[::2].copy()
                nw = rng.uniform(0.1, 3.0, len(new)) * 20.0
                nexp = np.where(np.arange(len(new)) % 2 == 0, now0 + 3 * W.NS, now0 + 600 * W.NS).astype(np.int64)
                eng.apply(W.rows_to_mask(upd, N), wv, gone, (new, None, nw, np.ones(len(new), np.int32), nexp))
                pos = np.searchsorted(upd, grow)
                hit = (pos < len(upd)) & (upd[np.minimum(pos, len(upd) - 1)] == grow)
                live = host["expiry_ns"] != W.RELEASED
                host["wants"] = np.where(hit & live, wv[np.minimum(pos, len(upd) - 1)], host["wants"])
                rel = np.isin(grow, gone)
                for k, v in (("has", 0.0), ("wants", 0.0), ("subclients", 0), ("expiry_ns", W.RELEASED)):
                    host[k] = np.where(rel, v, host[k])
                pos = np.searchsorted(new, grow)
                arr = (pos < len(new)) & (new[np.minimum(pos, len(new) - 1)] == grow)
                j = np.minimum(pos, len(new) - 1)
                host["has"] = np.where(arr, 0.0, host["has"])
                host["wants"] = np.where(arr, nw[j], host["wants"])
                host["subclients"] = np.where(arr, 1, host["subclients"])
                host["expiry_ns"] = np.where(arr, nexp[j], host["expiry_ns"])
                W.add_store_sums(host)
                assert arr.sum() > 0 and rel.sum() > 0 and hit.sum() > 0
            for now in seg:  # exactly bench.py's step: nothing read between the ticks
                eng.apportion(now, writeback=True, asynchronous=True, defer_join=True)
                _host_tick(host, now)
                ticks += 1
            eng.sync()
            _check(eng, host, pick, so, f"segment {si} ({ticks} ticks)")
        kt = eng.kernel_times()
        for k in ("large_spec", "large_redo", "subs_merged", "small_tiles"):
            assert kt.get(k, (0, 0))[0] >= 8, (k, kt)
        dense = sum(kt.get(n + "_dense", (0, 0))[0] for n in ("block128x4", "block128x8", "block256x8", "block2k4k"))
        rest = sum(kt.get(n + "_rest", (0, 0))[0] for n in ("block128x4", "block128x8", "block256x8", "block2k4k"))
        assert dense >= 20 and rest < dense, kt  # the dense kernels ran, most ticks without a rest kernel
        print(f"\nC2 full size: {ticks} back-to-back async ticks in 4 segments, {len(pick)} resources "
              f"({len(host['wants'])} rows) against the oracle; kernel launches "
              f"{ {k: v[0] for k, v in kt.items()} }")
    finally:
        eng.close()
