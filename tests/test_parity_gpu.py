"""Parity of the HIP path (through the C-ABI) against the CPU oracle.

Bar: expiries / counts bit-exact; gets within
1e-9 * max(|ref|, capacity_r); the wave-packed small-resource path is bit-exact
(it sums in the oracle's row order).  Full-size configs are checked on sampled
resources, which the oracle evaluates on the same rows.
"""
import json
import os

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import (assert_leases_match, assert_resources_match, binned_sizes, float_close, row_capacity,
                         snapshot_with_sizes)

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))
NOW = W.NOW_NS


@pytest.fixture(scope="module")
def eng():
    from doorman_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def run(eng, snap, writeback=False, recompute=False):
    eng.load(snap)
    eng.apportion(NOW, writeback=writeback, recompute=recompute)
    gets, exp = eng.leases()
    return gets, exp, eng.resources()


@pytest.mark.parametrize("case", KATS["snapshot"], ids=lambda c: c["name"])
def test_reference_kats_bit_exact(eng, case):
    n = len(case["wants"])
    snap = W.make_snapshot([n], case["wants"], case["has"], case["sub"], NOW + 300 * W.NS, case["kind"],
                           case["capacity"], lease_length_s=300)
    gets, exp, _ = run(eng, snap)
    assert gets.tolist() == case["gets"]
    assert (exp == NOW + 300 * W.NS).all()


@pytest.mark.parametrize("size", [3, 40, 200, 1000, 3000, 10000])
@pytest.mark.parametrize("kind", [2, 3])
def test_doc_examples_at_every_bin(eng, size, kind):
    """doc/algorithms.md:44-69 pattern replicated to each dispatch bin: one greedy
    client, one moderate, the rest below the equal share."""
    rng = np.random.default_rng(size)
    C = 120.0 * size / 3
    wants = np.full(size, 10.0 * C / 120.0 / (size / 3))
    wants[0], wants[1] = 1000.0 * C / 120, 50.0 * C / 120 / (size / 3)
    rng.shuffle(wants)
    snap = W.make_snapshot([size], wants, 0.0, 1, NOW + W.NS, kind, C)
    gets, exp, res = run(eng, snap)
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref)
    assert_resources_match(snap, res, ref)


@pytest.mark.parametrize("variant", ["uniform", "edge"])
def test_sub_wave_bins(eng, variant):
    """The sub-wave bins (9-256 rows: 8 x 2, 16 x 2, 16 x 4, 32 x 4, 64 x 4 lane groups)
    in their one launch (k_subs) match the oracle."""
    rng = np.random.default_rng(77)
    sizes = np.concatenate([binned_sizes(rng), rng.integers(9, 257, 300)])
    snap = snapshot_with_sizes(rng, sizes, edge=variant == "edge")
    eng.load(snap)
    eng.apportion(NOW)
    gets, exp = eng.leases()
    res = eng.resources()
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, variant)
    assert_resources_match(snap, res, ref, variant)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("variant", ["uniform", "hetero", "edge"])
@pytest.mark.parametrize("recompute", [False, True])
def test_random_all_bins(eng, seed, variant, recompute):
    rng = np.random.default_rng(1000 + seed)
    sizes = binned_sizes(rng)
    snap = snapshot_with_sizes(rng, sizes, hetero=variant == "hetero", edge=variant == "edge")
    if recompute:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            snap.pop(k)
    gets, exp, res = run(eng, snap, recompute=recompute)
    ref = O.apportion(snap, NOW)
    label = f"seed={seed} {variant} recompute={recompute}"
    assert_leases_match(snap, gets, exp, ref, label)
    assert_resources_match(snap, res, ref, label)


@pytest.mark.parametrize("seed", range(4))
def test_fair_share_heavy_contention(eng, seed):
    """Every resource FairShare, most clients above the equal share, some exactly at
    round thresholds: exercises round 2 (algorithm.go:188-204) in every bin."""
    rng = np.random.default_rng(2000 + seed)
    sizes = binned_sizes(rng, per_bin=2)
    snap = snapshot_with_sizes(rng, sizes, kinds=(3,), hetero=seed % 2 == 1, expired_frac=0.0, learning_frac=0.0,
                               parent_expired_frac=0.0)
    n_of_row = np.maximum(np.repeat(sizes, sizes), 1)
    cap = np.repeat(snap["capacity"], sizes)
    snap["wants"] = np.where(rng.random(len(n_of_row)) < 0.7, rng.uniform(1.0, 4.0, len(n_of_row)),
                             rng.uniform(0.0, 1.0, len(n_of_row))) * cap / n_of_row
    W.add_store_sums(snap)
    gets, exp, res = run(eng, snap)
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, f"seed={seed}")
    assert_resources_match(snap, res, ref)


@pytest.mark.parametrize("seed", range(3))
def test_scattered_small_resources_list_tiles(eng, seed):
    """Small resources interleaved with larger ones (runs shorter than kTileMinRun = 64,
    as in a store whose resource ids come in no size order) go to list tiles: each
    thread stages its own resource's rows.  The small resources' leases and sums are
    still bit-exact (row-order sums); long runs beside them keep the contiguous tiles."""
    rng = np.random.default_rng(3100 + seed)
    small = rng.integers(0, 5, 2000)
    other = rng.integers(5, 300, 2000)
    mix = np.where(rng.random(2000) < 0.5, small, other)
    sizes = np.concatenate([mix, rng.integers(1, 5, 700), mix[::-1]])  # a long run in the middle
    snap = snapshot_with_sizes(rng, sizes, hetero=seed == 1, edge=seed == 2)
    gets, exp, res = run(eng, snap)
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, f"seed={seed}")
    assert_resources_match(snap, res, ref)
    so = snap["seg_off"]
    sm = np.flatnonzero(np.diff(so) <= 4)
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in sm])
    assert float_close(gets[rows], ref["gets"][rows], 0.0, tol=0.0).all()
    for a, b in (("sum_has", "res_sum_has"), ("sum_wants", "res_sum_wants")):
        assert float_close(res[a][sm], ref[b][sm], 0.0, tol=0.0).all(), a
    info = eng.plan_info()
    assert info["small_tiles"] > 1


@pytest.mark.parametrize("seed", range(5))
def test_small_resources_bit_exact(eng, seed):
    """Resources of <= kSmallMax (4) rows go through the tiles' literal path, which
    sums in row order like the oracle: results are bit-identical, per-resource sums too."""
    rng = np.random.default_rng(3000 + seed)
    snap = snapshot_with_sizes(rng, rng.integers(0, 5, 3000), hetero=seed % 2 == 1, edge=seed >= 3)
    if seed == 2:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            snap.pop(k)
    gets, exp, res = run(eng, snap, recompute=seed == 2)
    ref = O.apportion(snap, NOW)
    np.testing.assert_array_equal(exp, ref["expiry_ns"])
    assert float_close(gets, ref["gets"], 0.0, tol=0.0).all()
    np.testing.assert_array_equal(res["count"], ref["res_count"])
    for a, b in (("sum_has", "res_sum_has"), ("sum_wants", "res_sum_wants"), ("safe_capacity", "res_safe_capacity")):
        assert float_close(res[a], ref[b], 0.0, tol=0.0).all(), a


def test_deterministic(eng):
    rng = np.random.default_rng(7)
    snap = snapshot_with_sizes(rng, binned_sizes(rng), hetero=True)
    g1, e1, r1 = run(eng, snap)
    g2, e2, r2 = run(eng, snap)
    assert g1.tobytes() == g2.tobytes() and e1.tobytes() == e2.tobytes()
    assert r1["sum_has"].tobytes() == r2["sum_has"].tobytes()


@pytest.mark.parametrize("cols", ["auto", "inplace", "alternate"])
def test_writeback_updates_store_like_assign(eng, cols):
    """DM_WRITEBACK: has := gets, expiry := now + lease, released rows zeroed and
    the running sums updated (store.go:142-167); a second tick on the written-back
    store matches the oracle on that store.  Both column modes (in place, and the
    alternate has/expiry pair that becomes the store's)."""
    rng = np.random.default_rng(11)
    snap = snapshot_with_sizes(rng, binned_sizes(rng), expired_frac=0.1)
    ref = O.apportion(snap, NOW)
    eng.load(snap)
    eng.apportion(NOW, writeback=True, wb_columns=cols)
    st = eng.read_store()
    live = ref["expiry_ns"] != W.RELEASED
    assert float_close(st["has"], np.where(live, ref["gets"], 0.0), np.repeat(snap["capacity"],
                       np.diff(snap["seg_off"]))).all()
    np.testing.assert_array_equal(st["expiry_ns"], ref["expiry_ns"])
    assert (st["wants"][~live] == 0).all() and (st["subclients"][~live] == 0).all()
    res = eng.resources()
    assert_resources_match(snap, res, ref)
    # second tick, later clock, on the device store as it now stands
    snap2 = dict(snap)
    snap2.update(has=st["has"], wants=st["wants"], subclients=st["subclients"], expiry_ns=st["expiry_ns"],
                 agg_count=res["count"], agg_sum_has=res["sum_has"], agg_sum_wants=res["sum_wants"])
    now2 = NOW + 200 * W.NS
    ref2 = O.apportion(snap2, now2)
    eng.apportion(now2, writeback=False)
    g2, e2 = eng.leases()
    assert_leases_match(snap2, g2, e2, ref2, "second tick")


def test_upsert_and_release(eng):
    """Assign / Release on the device store keep the running sums (store.go:142-167)."""
    rng = np.random.default_rng(12)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=False), expired_frac=0.0)
    eng.load(snap)
    N = len(snap["wants"])
    rows = rng.choice(N, N // 10, replace=False)
    new_w = rng.uniform(0, 50, len(rows))
    new_h = rng.uniform(0, 5, len(rows))
    new_s = np.ones(len(rows), np.int64)
    new_e = np.full(len(rows), NOW + 100 * W.NS)
    eng.upsert(rows, new_h, new_w, new_s, new_e)
    gone = rng.choice(np.setdiff1d(np.arange(N), rows), N // 20, replace=False)
    eng.release(gone)
    # the same edits applied to the host snapshot
    snap2 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    seg_of = np.repeat(np.arange(len(snap["seg_off"]) - 1), np.diff(snap["seg_off"]))
    for r, w, h, s, e in zip(rows, new_w, new_h, new_s, new_e):
        g = seg_of[r]
        snap2["agg_sum_has"][g] += h - snap2["has"][r]
        snap2["agg_sum_wants"][g] += w - snap2["wants"][r]
        snap2["agg_count"][g] += s - snap2["subclients"][r]
        snap2["has"][r], snap2["wants"][r], snap2["subclients"][r], snap2["expiry_ns"][r] = h, w, s, e
    for r in gone:
        g = seg_of[r]
        snap2["agg_sum_has"][g] -= snap2["has"][r]
        snap2["agg_sum_wants"][g] -= snap2["wants"][r]
        snap2["agg_count"][g] -= snap2["subclients"][r]
        snap2["has"][r] = snap2["wants"][r] = 0.0
        snap2["subclients"][r] = 0
        snap2["expiry_ns"][r] = W.RELEASED
    st = eng.read_store()
    np.testing.assert_array_equal(st["expiry_ns"], snap2["expiry_ns"])
    np.testing.assert_array_equal(st["wants"], snap2["wants"])
    agg = eng.resources(safe=False)
    np.testing.assert_array_equal(agg["count"], snap2["agg_count"])
    assert float_close(agg["sum_wants"], snap2["agg_sum_wants"], np.maximum(snap["capacity"], 1e3), 1e-12).all()
    eng.apportion(NOW)
    gets, exp = eng.leases()
    snap2["agg_sum_has"], snap2["agg_sum_wants"] = agg["sum_has"], agg["sum_wants"]
    ref = O.apportion(snap2, NOW)
    assert_leases_match(snap2, gets, exp, ref, "after upsert/release")


def test_proto_form(eng):
    """server.go:787-791: capacity, Expiry.Unix(), int64(RefreshInterval.Seconds())."""
    rng = np.random.default_rng(13)
    snap = snapshot_with_sizes(rng, np.array([5, 0, 70, 300]), expired_frac=0.2)
    gets, exp, _ = run(eng, snap)
    cap, exp_s, ref_s = eng.leases_proto()
    assert cap.tobytes() == gets.tobytes()
    live = exp != W.RELEASED
    np.testing.assert_array_equal(exp_s[live], exp[live] // W.NS)
    refresh_row = np.repeat(snap["refresh_interval_s"], np.diff(snap["seg_off"]))
    np.testing.assert_array_equal(ref_s[live], refresh_row[live])


def test_unknown_kind_rejected(eng):
    from doorman_amd._lib import DM_E_KIND, DmError
    snap = W.make_snapshot([2], [1.0, 2.0], 0.0, 1, NOW + W.NS, 9, 10.0)
    with pytest.raises(DmError) as e:
        eng.load(snap)
    assert e.value.code == DM_E_KIND


def _sample_check(eng, snap, resources, label):
    gets, exp = eng.leases()
    res = eng.resources()
    sub = W.subset(snap, resources)
    ref = O.apportion(sub, NOW)
    so = snap["seg_off"]
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in resources])
    assert_leases_match(sub, gets[rows], exp[rows], ref, label)
    assert_resources_match(sub, {k: v[resources] for k, v in res.items()}, ref, label)


@pytest.mark.parametrize("kind", [W.FAIR_SHARE, W.PROPORTIONAL_SHARE])
def test_c1_full_size_sampled(eng, kind):
    """configs[1]: 10k resources x 1k clients (10M leases), sampled against the oracle."""
    snap = W.c1(kind=kind)
    eng.load(snap)
    eng.apportion(NOW)
    rng = np.random.default_rng(5)
    _sample_check(eng, snap, np.sort(rng.choice(10_000, 48, replace=False)), f"C1 kind={kind}")


@pytest.mark.parametrize("recompute", [False, True])
def test_c1_writeback_ticks_dense_sampled(eng, recompute):
    """The bench's tick sequence at configs[1] size: back-to-back writeback ticks (from
    the second tick on every resource is dense, its subclients column not read);
    sampled resources match the oracle replaying the same ticks on a host copy, with
    the store's running sums or with sums rebuilt from the rows (DM_AGG_RECOMPUTE)."""
    snap = W.c1()
    eng.load(snap)
    rng = np.random.default_rng(8)
    resources = np.sort(rng.choice(10_000, 48, replace=False))
    host = W.subset(snap, resources)
    so = snap["seg_off"]
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in resources])
    for t in range(3):
        now = NOW + t * W.NS
        eng.apportion(now, writeback=True, recompute=recompute)
        gets, exp = eng.leases()
        ref = O.apportion(host, now)
        assert_leases_match(host, gets[rows], exp[rows], ref, f"C1 writeback tick {t} recompute={recompute}")
        live = ref["expiry_ns"] != W.RELEASED
        host["has"] = np.where(live, ref["gets"], 0.0)
        host["wants"] = np.where(live, host["wants"], 0.0)
        host["subclients"] = np.where(live, host["subclients"], 0)
        host["expiry_ns"] = ref["expiry_ns"].copy()
        W.add_store_sums(host)
        if t == 0:
            assert eng.store_stats()["dense_resources"] == 10_000
    res = eng.resources()
    assert_resources_match(host, {k: v[resources] for k, v in res.items()}, O.apportion(host, now), "C1 final")


def test_c2_zipf_full_size_sampled(eng):
    """configs[2]: 1M resources, Zipf 1..1M clients, mixed kinds, 5% learning."""
    snap = W.c2()
    eng.load(snap)
    info = eng.plan_info()
    assert info["leases"] == 13_970_034 and info["large_resources"] > 0 and info["small_tiles"] > 0
    eng.apportion(NOW)
    rng = np.random.default_rng(6)
    sample = np.unique(np.concatenate([[0, 1, 2, 3, 7, 100, 121, 122, 243, 244],
                                       rng.choice(1_000_000, 300, replace=False)]))
    _sample_check(eng, snap, sample, "C2")


def test_c3_full_size_sampled_and_checksum(eng):
    """configs[3] size on one GPU: 100M leases (4.4 GB table, the HBM-streaming load
    batching), FS/PS mixed with 1% expired rows.  Sampled resources against the
    oracle, and over all 100k resources a size-independent property: after a
    writeback tick each resource's sumHas equals the sum of its live leases' gets."""
    snap = W.uniform(100_000, 1_000, kind="mixed", seed=33, expired_frac=0.01)
    eng.load(snap)
    eng.apportion(NOW)
    rng = np.random.default_rng(7)
    _sample_check(eng, snap, np.sort(rng.choice(100_000, 24, replace=False)), "C3")
    eng.apportion(NOW, writeback=True)
    gets, exp = eng.leases()
    res = eng.resources(safe=False)
    live = exp != W.RELEASED
    per_res = np.add.reduceat(np.where(live, gets, 0.0), snap["seg_off"][:-1])
    np.testing.assert_allclose(res["sum_has"], per_res, rtol=0, atol=1e-9 * 1000.0)
    np.testing.assert_array_equal(res["count"], np.add.reduceat(live.astype(np.int64), snap["seg_off"][:-1]))
    del snap, gets, exp


@pytest.mark.parametrize("cols", ["inplace", "alternate"])
def test_streaming_rounds_match_oracle(eng, cols):
    """configs[4]'s loop at small size: per 5 s round, 10% wants updates, 1% departures,
    new clients into free rows, then a writeback tick (with Clean of leases that
    expired).  A host copy of the store receives the same updates and the tick's
    writeback; the oracle decides it each round from exact sums while the device
    uses its running sums."""
    rng = np.random.default_rng(44)
    snap = W.uniform(3000, 500, kind="mixed", seed=44)
    N = len(snap["wants"])
    free = rng.random(N) < 0.05
    snap["wants"][free] = 0.0
    snap["has"][free] = 0.0
    snap["subclients"] = np.where(free, 0, 1).astype(np.int64)
    snap["expiry_ns"][free] = W.RELEASED
    W.add_store_sums(snap)
    eng.load(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    now = NOW
    for rnd in range(6):
        now += 5 * W.NS
        alive = np.flatnonzero(host["expiry_ns"] != W.RELEASED)
        upd = np.sort(rng.choice(alive, len(alive) // 10, replace=False))
        w = rng.uniform(0.5, 1.5, len(upd)) * 2.0
        eng.update_wants(upd, w)
        host["wants"][upd] = w
        rest = np.setdiff1d(alive, upd)
        gone = np.sort(rng.choice(rest, len(alive) // 100, replace=False))
        eng.release(gone)
        for k, v in (("wants", 0.0), ("has", 0.0), ("subclients", 0), ("expiry_ns", W.RELEASED)):
            host[k][gone] = v
        pool = np.flatnonzero(host["expiry_ns"] == W.RELEASED)
        new = np.sort(rng.choice(pool, min(len(pool), len(gone)), replace=False))
        nw = rng.uniform(0.5, 1.5, len(new))
        ne = np.full(len(new), now + 600 * W.NS)
        eng.upsert(new, np.zeros(len(new)), nw, np.ones(len(new), np.int64), ne)
        host["wants"][new], host["has"][new], host["subclients"][new], host["expiry_ns"][new] = nw, 0.0, 1, ne
        W.add_store_sums(host)
        eng.apportion(now, writeback=True, wb_columns=cols)
        gets, exp = eng.leases()
        ref = O.apportion(host, now)
        assert_leases_match(host, gets, exp, ref, f"round {rnd}")
        live = ref["expiry_ns"] != W.RELEASED  # the tick's writeback, on the host copy
        host["has"] = np.where(live, ref["gets"], 0.0)
        host["wants"] = np.where(live, host["wants"], 0.0)
        host["subclients"] = np.where(live, host["subclients"], 0)
        host["expiry_ns"] = ref["expiry_ns"].copy()
    store = eng.read_store()
    np.testing.assert_array_equal(store["subclients"], host["subclients"])
    np.testing.assert_array_equal(store["expiry_ns"], host["expiry_ns"])


@pytest.mark.parametrize("case", [c for c in KATS["server"] if "error" not in c and "release" not in c],
                         ids=lambda c: c["name"])
def test_server_kats_through_the_abi(eng, case):
    """server_test.go:339-553 (learning mode 20/90/100, learning persists across
    LoadConfig, GetServerCapacity bands -> 100) as one-client ticks on the device."""
    from test_oracle_golden import server_kat_snapshots
    for snap, expect in server_kat_snapshots(case):
        gets, exp, _ = run(eng, snap)
        assert gets[0] == expect


def test_wrong_number_of_clients_through_the_abi():
    """server_test.go:483-503: num_clients < 1 is codes.InvalidArgument."""
    from doorman_amd._lib import DM_E_ARGUMENT, DmError
    from doorman_amd.engine import aggregate_bands
    with pytest.raises(DmError) as e:
        aggregate_bands([10.0], [0])
    assert e.value.code == DM_E_ARGUMENT


def test_lease_length_and_refresh_interval_through_the_abi(eng):
    """algorithm_test.go:285-312: expiry = now + lease_length, refresh as configured."""
    k = KATS["lease_length"]
    snap = W.make_snapshot([1], [k["wants"]], [0.0], [k["sub"]], NOW + W.NS, k["kind"], k["capacity"],
                           k["lease_length"], k["refresh_interval"])
    run(eng, snap)
    cap, exp_s, ref_s = eng.leases_proto()
    assert exp_s[0] - NOW // W.NS == k["expiry_minus_now_s"]
    assert ref_s[0] == k["refresh_s"]


def test_insert_new_clients_into_free_slots(eng):
    """New clients: a store keeps released rows (tombstones) as free slots; an upsert
    onto one is LeaseStore.Assign of a new client (store.go:153-167: sums += new - 0)."""
    rng = np.random.default_rng(21)
    sizes = binned_sizes(rng, large=True)
    snap = snapshot_with_sizes(rng, sizes, expired_frac=0.0, kinds=(2, 3))
    N = len(snap["wants"])
    free = rng.choice(N, N // 8, replace=False)  # slack rows, released
    for k in ("wants", "has"):
        snap[k][free] = 0.0
    snap["subclients"][free] = 0
    snap["expiry_ns"][free] = W.RELEASED
    W.add_store_sums(snap)
    eng.load(snap)
    new = rng.choice(free, len(free) // 2, replace=False)
    seg_of = np.repeat(np.arange(len(sizes)), sizes)
    cap_row = snap["capacity"][seg_of[new]]
    n_row = np.maximum(sizes[seg_of[new]], 1)
    w = rng.uniform(0, 2, len(new)) * cap_row / n_row
    h = np.zeros(len(new))
    s = np.ones(len(new), np.int64)
    e = np.full(len(new), NOW + 60 * W.NS)
    eng.upsert(new, h, w, s, e)
    snap2 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    snap2["wants"][new], snap2["has"][new], snap2["subclients"][new], snap2["expiry_ns"][new] = w, h, s, e
    np.add.at(snap2["agg_sum_wants"], seg_of[new], w)
    np.add.at(snap2["agg_count"], seg_of[new], s)
    agg = eng.resources(safe=False)
    np.testing.assert_array_equal(agg["count"], snap2["agg_count"])
    snap2["agg_sum_wants"], snap2["agg_sum_has"] = agg["sum_wants"], agg["sum_has"]
    eng.apportion(NOW)
    gets, exp = eng.leases()
    ref = O.apportion(snap2, NOW)
    assert_leases_match(snap2, gets, exp, ref, "after inserts")
    assert (exp[np.setdiff1d(free, new)] == W.RELEASED).all()


def test_upsert_rejects_duplicate_and_out_of_range_rows(eng):
    from doorman_amd._lib import DM_E_INVAL, DM_E_RANGE, DmError
    snap = W.make_snapshot([4, 4], np.ones(8), np.zeros(8), 1, NOW + W.NS, 3, 10.0)
    eng.load(snap)
    one = np.ones(2)
    with pytest.raises(DmError) as e:
        eng.upsert([1, 1], one, one, [1, 1], [NOW, NOW])
    assert e.value.code == DM_E_INVAL
    with pytest.raises(DmError) as e:
        eng.upsert([1, 8], one, one, [1, 1], [NOW, NOW])
    assert e.value.code == DM_E_RANGE


def test_rejected_update_leaves_store_untouched(eng):
    """Validation runs on the device before the apply kernel: duplicate, out-of-range
    rows and bad subclients reject the whole call; the store and its sums are unchanged
    and the row bitmap is clean for the next call."""
    from doorman_amd._lib import DM_E_INVAL, DM_E_RANGE, DmError
    snap = W.make_snapshot([4, 4], np.ones(8), np.zeros(8), 1, NOW + W.NS, 3, 10.0)
    eng.load(snap)
    before = eng.read_store()
    for call, code in [(lambda: eng.update_wants([0, 5, 5], [2.0, 2.0, 2.0]), DM_E_INVAL),
                       (lambda: eng.update_wants([0, 9], [2.0, 2.0]), DM_E_RANGE),
                       (lambda: eng.release([3, -1]), DM_E_RANGE),
                       (lambda: eng.upsert([2], [1.0], [1.0], [-3], [NOW]), DM_E_INVAL),
                       (lambda: eng.upsert([2, 6], [1.0, 1.0], [1.0, 1.0], [1, 2 ** 31], [NOW, NOW]), DM_E_INVAL)]:
        with pytest.raises(DmError) as e:
            call()
        assert e.value.code == code
        after = eng.read_store()
        for k in before:
            np.testing.assert_array_equal(before[k], after[k], err_msg=k)
    # the same rows are accepted afterwards (bitmap cleared), unsorted order is fine
    eng.update_wants([5, 0], [3.0, 4.0])
    assert eng.read_store()["wants"][[0, 5]].tolist() == [4.0, 3.0]


def test_pinned_update_buffers(eng):
    """dm_host_alloc buffers feed the update calls like ordinary host arrays."""
    rng = np.random.default_rng(5)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=False), expired_frac=0.0, kinds=(2, 3))
    eng.load(snap)
    N = len(snap["wants"])
    n = N // 7
    rows = eng.host_empty(n, np.int64)
    rows[:] = np.sort(rng.choice(N, n, replace=False))
    w = eng.host_empty(n)
    w[:] = snap["wants"][rows] * rng.uniform(0.5, 2.0, n)
    eng.update_wants(rows, w)
    snap2 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    snap2["wants"][rows] = w
    snap2["agg_sum_wants"] = eng.resources(safe=False)["sum_wants"]
    eng.apportion(NOW)
    gets, exp = eng.leases()
    assert_leases_match(snap2, gets, exp, O.apportion(snap2, NOW), "pinned update")


def test_update_wants_narrow_assign(eng):
    """dm_store_update_wants: Assign of a refresh that changes only wants."""
    rng = np.random.default_rng(22)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=True), expired_frac=0.0, kinds=(2, 3))
    eng.load(snap)
    N = len(snap["wants"])
    rows = rng.choice(N, N // 5, replace=False)
    neww = snap["wants"][rows] * rng.uniform(0.5, 2.0, len(rows))
    eng.update_wants(rows, neww)
    snap2 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    seg_of = np.repeat(np.arange(len(snap["seg_off"]) - 1), np.diff(snap["seg_off"]))
    np.add.at(snap2["agg_sum_wants"], seg_of[rows], neww - snap["wants"][rows])
    snap2["wants"][rows] = neww
    agg = eng.resources(safe=False)
    assert float_close(agg["sum_wants"], snap2["agg_sum_wants"], np.maximum(snap["capacity"], 1.0), 1e-12).all()
    snap2["agg_sum_wants"] = agg["sum_wants"]
    eng.apportion(NOW)
    gets, exp = eng.leases()
    assert_leases_match(snap2, gets, exp, O.apportion(snap2, NOW), "after update_wants")


@pytest.mark.parametrize("cols", ["inplace", "alternate"])
def test_deferred_join_matches_joined_ticks(eng, cols):
    """DM_DEFER_JOIN: back-to-back asynchronous writeback ticks whose work classes
    stay on the auxiliary streams (no per-tick join) leave bit for bit the store,
    running sums and leases of the same ticks run with a join per tick; then a
    store update between deferred ticks (the call joins first) and two more ticks
    agree too (to the ULP of the update's atomically accumulated running sums)."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(21)
    snap = snapshot_with_sizes(rng, binned_sizes(rng), expired_frac=0.05)
    N = len(snap["wants"])
    upd = np.sort(rng.choice(N, N // 8, replace=False))
    new_w = rng.uniform(0.0, 50.0, len(upd))
    cap = np.repeat(snap["capacity"], np.diff(snap["seg_off"]))
    other = Engine(0)

    def ticks(e, defer, t0, n):
        for t in range(t0, t0 + n):
            e.apportion(NOW + t * W.NS, writeback=True, asynchronous=True, wb_columns=cols, defer_join=defer)

    def state(e):
        gets, exp = e.leases()
        return gets, exp, e.read_store(), e.resources(safe=False)

    try:
        outs = []
        for e, defer in ((eng, True), (other, False)):
            e.load(snap)
            ticks(e, defer, 0, 6)
            outs.append(state(e))
        (g1, e1, s1, r1), (g2, e2, s2, r2) = outs
        assert g1.tobytes() == g2.tobytes() and e1.tobytes() == e2.tobytes()
        for k in ("has", "wants", "subclients", "expiry_ns"):
            assert s1[k].tobytes() == s2[k].tobytes(), k
        for k in ("count", "sum_has", "sum_wants"):
            assert r1[k].tobytes() == r2[k].tobytes(), k
        outs = []
        for e, defer in ((eng, True), (other, False)):
            ticks(e, defer, 6, 1)
            e.update_wants(upd, new_w)
            ticks(e, defer, 7, 2)
            outs.append(state(e))
        (g1, e1, s1, r1), (g2, e2, s2, r2) = outs
        assert float_close(g1, g2, cap, 1e-12).all()
        np.testing.assert_array_equal(e1, e2)
        assert s1["wants"].tobytes() == s2["wants"].tobytes()
        np.testing.assert_array_equal(r1["count"], r2["count"])
        assert float_close(r1["sum_wants"], r2["sum_wants"], np.maximum(snap["capacity"], 1.0), 1e-12).all()
        # and the deferred store agrees with the oracle on one more tick
        ref_snap = dict(snap)
        ref_snap.update(has=s1["has"], wants=s1["wants"], subclients=s1["subclients"], expiry_ns=s1["expiry_ns"],
                        agg_count=r1["count"], agg_sum_has=r1["sum_has"], agg_sum_wants=r1["sum_wants"])
        now = NOW + 10 * W.NS
        eng.apportion(now, asynchronous=True, defer_join=True)
        gets, exp = eng.leases()  # joins
        assert_leases_match(ref_snap, gets, exp, O.apportion(ref_snap, now), "after deferred ticks")
    finally:
        other.close()


def test_update_wants_mask_matches_row_form(eng):
    """dm_store_update_wants_mask (rows as a bit mask, values packed in row order)
    leaves the store and running sums of dm_store_update_wants on the same rows,
    across resource boundaries inside a 64-row word and for a window that starts
    at a 64-row boundary; the next tick matches the oracle."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(31)
    snap = snapshot_with_sizes(rng, binned_sizes(rng), expired_frac=0.0)
    N = len(snap["wants"])
    cap = np.maximum(snap["capacity"], 1.0)
    other = Engine(0)
    try:
        eng.load(snap)
        other.load(snap)
        rows = np.sort(rng.choice(N, N // 7, replace=False))
        w = rng.uniform(0.0, 40.0, len(rows))
        eng.update_wants_mask(W.rows_to_mask(rows, N), w)
        other.update_wants(rows, w)
        lo = 64 * (N // 128)
        sub = np.sort(rng.choice(np.arange(lo, N), (N - lo) // 3, replace=False))
        w2 = rng.uniform(0.0, 40.0, len(sub))
        eng.update_wants_mask(W.rows_to_mask(sub, N - lo, first_row=lo), w2, first_row=lo)
        other.update_wants(sub, w2)
        s1, s2 = eng.read_store(), other.read_store()
        assert s1["wants"].tobytes() == s2["wants"].tobytes()
        r1, r2 = eng.resources(safe=False), other.resources(safe=False)
        np.testing.assert_array_equal(r1["count"], r2["count"])
        assert float_close(r1["sum_wants"], r2["sum_wants"], cap, 1e-12).all()
        exact = snap["agg_sum_wants"].copy()
        np.add.at(exact, np.repeat(np.arange(len(cap)), np.diff(snap["seg_off"])), s1["wants"] - snap["wants"])
        assert float_close(r1["sum_wants"], exact, cap, 1e-12).all()
        ref_snap = dict(snap)
        ref_snap.update(wants=s1["wants"], agg_sum_wants=r1["sum_wants"])
        eng.apportion(NOW)
        gets, exp = eng.leases()
        assert_leases_match(ref_snap, gets, exp, O.apportion(ref_snap, NOW), "after masked update")
    finally:
        other.close()


@pytest.mark.parametrize("form", ["rows", "mask"])
def test_wants_refresh_leaves_released_rows_alone(eng, form):
    """A released row is a free slot, not a client: a wants refresh naming it changes
    neither the row nor its resource's running sums (a returning client is an arrival,
    dm_store_upsert).  Written into the row, the wants would be subtracted from the
    running sum again by every later tick's Clean.  After refreshes that mix live and
    released rows, over several writeback ticks, every resource's sumWants equals the
    sum of its live rows' wants and its Count their subclients; each tick matches the
    oracle on the store as it stood."""
    rng = np.random.default_rng(4711)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=True), expired_frac=0.1, kinds=(2, 3),
                               learning_frac=0.0, parent_expired_frac=0.0)
    so = np.asarray(snap["seg_off"])
    N, R = len(snap["wants"]), len(so) - 1
    seg_of = np.repeat(np.arange(R), np.diff(so))
    cap = np.maximum(snap["capacity"], 1.0)
    eng.load(snap)
    now = NOW
    eng.apportion(now, writeback=True)  # the expired rows are released
    for t in range(4):
        st = eng.read_store()
        released = st["expiry_ns"] == W.RELEASED
        assert released.any()
        rows = np.sort(rng.choice(N, N // 6, replace=False))
        w = rng.uniform(0.0, 40.0, len(rows))
        if form == "rows":
            eng.update_wants(rows, w)
        else:
            eng.update_wants_mask(W.rows_to_mask(rows, N), w)
        st2 = eng.read_store()
        want_w = st["wants"].copy()
        live_rows = ~released[rows]
        want_w[rows[live_rows]] = w[live_rows]
        assert st2["wants"].tobytes() == want_w.tobytes(), f"round {t}: store wants"
        res = eng.resources(safe=False)
        live_w = np.where(released, 0.0, st2["wants"])
        assert float_close(res["sum_wants"], np.bincount(seg_of, live_w, R), cap, 1e-12).all(), f"round {t}"
        cur = dict(snap)
        cur.update(has=st2["has"], wants=st2["wants"], subclients=st2["subclients"], expiry_ns=st2["expiry_ns"],
                   agg_count=res["count"], agg_sum_has=res["sum_has"], agg_sum_wants=res["sum_wants"])
        now += 5 * W.NS
        ref = O.apportion(cur, now)
        eng.apportion(now, writeback=True)
        st3 = eng.read_store()
        live = ref["expiry_ns"] != W.RELEASED
        assert float_close(np.where(live, st3["has"], 0.0), np.where(live, ref["gets"], 0.0), row_capacity(cur)).all()
        res = eng.resources(safe=False)
        rel3 = st3["expiry_ns"] == W.RELEASED
        np.testing.assert_array_equal(res["count"], np.bincount(seg_of, np.where(rel3, 0, st3["subclients"]), R))
        assert float_close(res["sum_wants"], np.bincount(seg_of, np.where(rel3, 0.0, st3["wants"]), R), cap,
                           1e-12).all(), f"round {t}: after the tick"


def test_update_wants_mask_rejects_bad_input(eng):
    """Count mismatch (DM_E_INVAL), a bit past the store's end (DM_E_RANGE), a window
    not on a 64-row boundary (DM_E_INVAL): the store is left untouched."""
    from doorman_amd._lib import DM_E_INVAL, DM_E_RANGE, DmError
    rng = np.random.default_rng(32)
    snap = snapshot_with_sizes(rng, np.array([5, 70, 300]), expired_frac=0.0)
    N = len(snap["wants"])
    assert N % 64 != 0
    eng.load(snap)
    before, res0 = eng.read_store(), eng.resources(safe=False)
    mask = W.rows_to_mask([1, 5, 9], N)
    with pytest.raises(DmError) as e:
        eng.update_wants_mask(mask, [1.0, 2.0])
    assert e.value.code == DM_E_INVAL
    bad = mask.copy()
    bad[-1] |= np.uint64(1) << np.uint64(63)
    with pytest.raises(DmError) as e:
        eng.update_wants_mask(bad, [1.0, 2.0, 3.0, 4.0])
    assert e.value.code == DM_E_RANGE
    with pytest.raises(DmError) as e:
        eng.update_wants_mask(mask, [1.0, 2.0, 3.0], first_row=3)
    assert e.value.code == DM_E_INVAL
    after, res1 = eng.read_store(), eng.resources(safe=False)
    assert after["wants"].tobytes() == before["wants"].tobytes()
    assert res1["sum_wants"].tobytes() == res0["sum_wants"].tobytes()


def _round_parts(rng, snap):
    N = len(snap["wants"])
    alive = np.flatnonzero(snap["expiry_ns"] != W.RELEASED)
    upd = np.sort(rng.choice(alive, len(alive) // 9, replace=False))
    rest = np.setdiff1d(alive, upd)
    gone = np.sort(rng.choice(rest, len(alive) // 50, replace=False))
    new = np.sort(rng.choice(np.setdiff1d(np.arange(N), np.concatenate([upd, gone])), len(gone), replace=False))
    k = len(new)
    ups = (new, rng.uniform(0, 2, k), rng.uniform(0.5, 1.5, k), np.ones(k, np.int64), np.full(k, NOW + 900 * W.NS))
    return upd, rng.uniform(0.5, 1.5, len(upd)), gone, ups


def test_store_apply_matches_sequential_calls(eng):
    """dm_store_apply (refresh mask + departures + arrivals in one call, copies back
    to back) leaves the store of the three single calls; the next tick matches the
    oracle."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(41)
    snap = snapshot_with_sizes(rng, binned_sizes(rng), expired_frac=0.0)
    N = len(snap["wants"])
    cap = np.maximum(snap["capacity"], 1.0)
    upd, w, gone, ups = _round_parts(rng, snap)
    other = Engine(0)
    try:
        eng.load(snap)
        other.load(snap)
        eng.apply(W.rows_to_mask(upd, N), w, gone, ups)
        other.update_wants(upd, w)
        other.release(gone)
        other.upsert(*ups)
        s1, s2 = eng.read_store(), other.read_store()
        for k in ("has", "wants", "subclients", "expiry_ns"):
            assert s1[k].tobytes() == s2[k].tobytes(), k
        r1, r2 = eng.resources(safe=False), other.resources(safe=False)
        np.testing.assert_array_equal(r1["count"], r2["count"])
        for k in ("sum_has", "sum_wants"):
            assert float_close(r1[k], r2[k], cap, 1e-12).all(), k
        ref_snap = dict(snap)
        ref_snap.update(has=s1["has"], wants=s1["wants"], subclients=s1["subclients"], expiry_ns=s1["expiry_ns"],
                        agg_count=r1["count"], agg_sum_has=r1["sum_has"], agg_sum_wants=r1["sum_wants"])
        eng.apportion(NOW)
        gets, exp = eng.leases()
        assert_leases_match(ref_snap, gets, exp, O.apportion(ref_snap, NOW), "after dm_store_apply")
    finally:
        other.close()


def test_store_apply_chunked_refresh_matches_sequential_calls(eng):
    """A refresh of more than 2^23 values crosses PCIe in four chunks, each applied as it
    lands (dm_store_apply): the same store as dm_store_update_wants_mask + release +
    upsert one after another (wants bit for bit, sums within 1e-12), with updated rows
    in every chunk and in every resource, departures and arrivals after them, and a
    refreshed row that also departs (the departure wins in both)."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(43)
    sizes = rng.integers(700, 1300, 10_000)
    N = int(sizes.sum())
    snap = W.make_snapshot(sizes, rng.uniform(0.5, 2.0, N), rng.uniform(0.0, 1.0, N), 1,
                           np.full(N, NOW + 600 * W.NS), W.FAIR_SHARE, 1000.0)
    cap = np.maximum(snap["capacity"], 1.0)
    upd = np.arange(1, N, 1, dtype=np.int64)[rng.random(N - 1) < 0.9]  # ~9M values: four chunks
    assert len(upd) > 4 << 21
    w = rng.uniform(0.5, 1.5, len(upd))
    gone = np.sort(rng.choice(upd, 20_000, replace=False))  # refreshed, then departing
    free = np.setdiff1d(np.arange(N), upd)[:5000]
    k = len(free)
    ups = (free, None, rng.uniform(0.5, 1.5, k), np.ones(k, np.int64), np.full(k, NOW + 900 * W.NS))
    other = Engine(0)
    try:
        eng.load(snap)
        other.load(snap)
        eng.apply(W.rows_to_mask(upd, N), w, gone, ups, now_ns=NOW)
        other.update_wants_mask(W.rows_to_mask(upd, N), w)
        other.release(gone)
        other.upsert(free, np.zeros(k), ups[2], ups[3], ups[4])
        s1, s2 = eng.read_store(), other.read_store()
        for key in ("has", "wants", "subclients", "expiry_ns"):
            assert s1[key].tobytes() == s2[key].tobytes(), key
        r1, r2 = eng.resources(safe=False), other.resources(safe=False)
        np.testing.assert_array_equal(r1["count"], r2["count"])
        for key in ("sum_has", "sum_wants"):
            assert float_close(r1[key], r2[key], cap, 1e-12).all(), key
        live = s1["expiry_ns"] != W.RELEASED
        want = snap["wants"].copy()
        want[upd] = w
        want[gone] = 0.0
        want[free] = ups[2]
        assert s1["wants"][live].tobytes() == want[live].tobytes()
    finally:
        other.close()


def test_store_apply_stops_at_the_first_rejected_part(eng):
    """A rejected part (duplicate departure rows) returns its error; the refresh before
    it stays applied, the arrivals after it are not; a bad mask rejects everything."""
    from doorman_amd._lib import DM_E_INVAL, DmError
    rng = np.random.default_rng(42)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=False), expired_frac=0.0)
    N = len(snap["wants"])
    upd, w, gone, ups = _round_parts(rng, snap)
    eng.load(snap)
    before = eng.read_store()
    with pytest.raises(DmError) as e:
        eng.apply(W.rows_to_mask(upd, N), w, np.concatenate([gone, gone[:1]]), ups)
    assert e.value.code == DM_E_INVAL and "release" in str(e.value)
    st = eng.read_store()
    exp_w = before["wants"].copy()
    exp_w[upd] = w
    assert st["wants"].tobytes() == exp_w.tobytes()  # refresh applied, arrivals' wants not
    assert st["expiry_ns"].tobytes() == before["expiry_ns"].tobytes()  # no departure, no arrival
    eng.load(snap)
    with pytest.raises(DmError) as e:
        eng.apply(W.rows_to_mask(upd, N), w[:-1], gone, ups)
    assert e.value.code == DM_E_INVAL
    st = eng.read_store()
    for k in ("has", "wants", "subclients", "expiry_ns"):
        assert st[k].tobytes() == before[k].tobytes(), k


def test_c4_rounds_async_back_to_back(eng):
    """bench.py's C4 step with nothing read in between: five rounds of
    dm_store_apply_async + an asynchronous writeback tick enqueued back to back (two
    batches in flight, each batch's copies overlapping the tick before it), then the
    store and the last tick's leases those of the same rounds through the synchronous
    dm_store_apply on another context: wants, subclients, expiries and the running
    Count bit for bit; has, gets and the running sums within 1e-12 of capacity (the
    sums' updates are atomic adds, so their rounding order differs between contexts)."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(405)
    snap = _c4_store(rng, 2000, 300)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    so = snap["seg_off"]
    rounds, now = [], NOW
    for _ in range(5):
        now += 5 * W.NS
        mask, w, gone, new, nh, nw, ns, ne, upd = _c4_round(rng, host, now)
        ne = now + snap["lease_length_s"][np.searchsorted(so, new, side="right") - 1] * W.NS
        _apply_host(host, upd, w, gone, new, nh, nw, ns, ne)
        rounds.append((mask, w, gone, (new, None, nw, ns.astype(np.int32), None), now))
    other = Engine(0)
    try:
        eng.load(snap)
        other.load(snap)
        for mask, w, gone, ups, t in rounds:
            eng.apply(mask, w, gone, ups, now_ns=t, asynchronous=True)
            eng.apportion(t, writeback=True, asynchronous=True)
            other.apply(mask, w, gone, ups, now_ns=t)
            other.apportion(t, writeback=True)
        eng.apply_wait()
        s1, s2 = eng.read_store(), other.read_store()
        for k in ("wants", "subclients", "expiry_ns"):
            assert s1[k].tobytes() == s2[k].tobytes(), k
        cap_row = np.repeat(np.maximum(snap["capacity"], 1.0), np.diff(so))
        assert float_close(s1["has"], s2["has"], cap_row, 1e-12).all()
        r1, r2 = eng.resources(safe=False), other.resources(safe=False)
        np.testing.assert_array_equal(r1["count"], r2["count"])
        for k in ("sum_has", "sum_wants"):
            assert float_close(r1[k], r2[k], np.maximum(snap["capacity"], 1.0), 1e-12).all(), k
        g1, e1 = eng.leases()
        g2, e2 = other.leases()
        assert e1.tobytes() == e2.tobytes()
        assert float_close(g1, g2, cap_row, 1e-12).all()
    finally:
        other.close()


def test_store_apply_async_between_synchronous_calls_and_a_reload(eng):
    """Asynchronous batches interleaved with the synchronous update calls (which stage
    through their own buffers, stream-ordered after the batches) leave the store those
    calls leave in the same order on another context; a store load while a batch is in
    flight waits for it and then holds exactly the new snapshot."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(44)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=False), expired_frac=0.0)
    N = len(snap["wants"])
    upd, w, gone, ups = _round_parts(rng, snap)
    used = np.concatenate([upd, gone, ups[0]])
    extra = np.setdiff1d(np.arange(1, N, 5), used)[:2000]
    w_extra = rng.uniform(0.5, 1.5, len(extra))
    upd2 = np.setdiff1d(np.arange(2, N, 9), np.concatenate([used, extra]))
    w2 = rng.uniform(0.5, 1.5, len(upd2))
    other = Engine(0)
    try:
        eng.load(snap)
        other.load(snap)
        eng.apply(W.rows_to_mask(upd, N), w, gone, ups, asynchronous=True)
        eng.update_wants(extra, w_extra)
        eng.apply(W.rows_to_mask(upd2, N), w2, asynchronous=True)
        other.apply(W.rows_to_mask(upd, N), w, gone, ups)
        other.update_wants(extra, w_extra)
        other.apply(W.rows_to_mask(upd2, N), w2)
        s1, s2 = eng.read_store(), other.read_store()
        for k in ("has", "wants", "subclients", "expiry_ns"):
            assert s1[k].tobytes() == s2[k].tobytes(), k
        r1, r2 = eng.resources(safe=False), other.resources(safe=False)
        np.testing.assert_array_equal(r1["count"], r2["count"])
        for k in ("sum_has", "sum_wants"):
            assert float_close(r1[k], r2[k], np.maximum(snap["capacity"], 1.0), 1e-12).all(), k
        eng.apply_wait()
        eng.apply(W.rows_to_mask(upd, N), w, gone, ups, asynchronous=True)
        eng.load(snap)  # waits for the batch, then replaces the store
        st = eng.read_store()
        for k in ("wants", "has"):
            assert st[k].tobytes() == np.asarray(snap[k], np.float64).tobytes(), k
        eng.apply_wait()  # nothing left in flight
    finally:
        other.close()


def test_store_apply_async_reports_a_rejected_batch_later(eng):
    """dm_store_apply_async: a batch with a rejected part (duplicate departure rows) is
    enqueued without an error; the call that retires it (apply_wait) raises, naming the
    earlier asynchronous batch and its part.  The store then holds what dm_store_apply
    leaves for the same batch (its refresh, no departure, no arrival) plus a valid batch
    enqueued after it (rows bit for bit, sums within 1e-12); a clean batch retires
    without an error."""
    from doorman_amd._lib import DM_E_INVAL, DmError
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(42)
    snap = snapshot_with_sizes(rng, binned_sizes(rng, large=False), expired_frac=0.0)
    N = len(snap["wants"])
    upd, w, gone, ups = _round_parts(rng, snap)
    upd2 = np.setdiff1d(np.arange(0, N, 7), np.concatenate([gone, ups[0]]))
    w2 = rng.uniform(0.5, 1.5, len(upd2))
    other = Engine(0)
    try:
        eng.load(snap)
        other.load(snap)
        eng.apply(W.rows_to_mask(upd, N), w, np.concatenate([gone, gone[:1]]), ups, asynchronous=True)
        eng.apply(W.rows_to_mask(upd2, N), w2, asynchronous=True)  # a valid batch after it
        with pytest.raises(DmError) as e:
            eng.apply_wait()
        assert e.value.code == DM_E_INVAL and "earlier asynchronous batch" in str(e.value)
        assert "release" in str(e.value)
        with pytest.raises(DmError):
            other.apply(W.rows_to_mask(upd, N), w, np.concatenate([gone, gone[:1]]), ups)
        other.apply(W.rows_to_mask(upd2, N), w2)
        s1, s2 = eng.read_store(), other.read_store()
        for k in ("has", "wants", "subclients", "expiry_ns"):
            assert s1[k].tobytes() == s2[k].tobytes(), k
        r1, r2 = eng.resources(safe=False), other.resources(safe=False)
        np.testing.assert_array_equal(r1["count"], r2["count"])
        for k in ("sum_has", "sum_wants"):  # (atomic adds: the rounding order may differ)
            assert float_close(r1[k], r2[k], np.maximum(snap["capacity"], 1.0), 1e-12).all(), k
        eng.apply(W.rows_to_mask(upd2, N), w2, asynchronous=True)
        eng.apply_wait()  # nothing rejected
    finally:
        other.close()


@pytest.mark.parametrize("cols", ["inplace", "alternate"])
def test_follower_expiry_encoding(eng, cols):
    """A writeback tick leaves every lease a follower of its resource's expiry (only
    gets move per lease, include/doorman_hip.h): followers expire together when no
    tick refreshes them, rows upserted in between keep their own expiry, released
    rows stay released; leases, the store read back and the next ticks match the
    oracle on a host copy that stores every expiry explicitly."""
    rng = np.random.default_rng(91)
    sizes = binned_sizes(rng, per_bin=2)
    snap = snapshot_with_sizes(rng, sizes, kinds=(0, 1, 2, 3), expired_frac=0.05, learning_frac=0.1)
    snap["lease_length_s"] = np.where(rng.random(len(sizes)) < 0.5, 10, 400).astype(np.int64)
    eng.load(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    N = len(host["wants"])
    for rnd, dt in enumerate([0, 5, 25, 30, 31]):  # the 10-s resources' followers lapse at +25
        now = NOW + dt * W.NS
        if rnd == 3:  # explicit rows between ticks: refreshed leases with their own expiry
            rows = np.sort(rng.choice(N, N // 20, replace=False))
            nw = rng.uniform(0.0, 2.0, len(rows))
            ne = now + rng.integers(-3, 60, len(rows)) * W.NS
            eng.upsert(rows, np.zeros(len(rows)), nw, np.ones(len(rows), np.int64), ne)
            host["wants"][rows], host["has"][rows], host["subclients"][rows], host["expiry_ns"][rows] = nw, 0.0, 1, ne
            W.add_store_sums(host)
        eng.apportion(now, writeback=True, wb_columns=cols)
        gets, exp = eng.leases()
        ref = O.apportion(host, now)
        assert_leases_match(host, gets, exp, ref, f"tick {rnd}")
        live = ref["expiry_ns"] != W.RELEASED
        host["has"] = np.where(live, ref["gets"], 0.0)
        host["wants"] = np.where(live, host["wants"], 0.0)
        host["subclients"] = np.where(live, host["subclients"], 0)
        host["expiry_ns"] = ref["expiry_ns"].copy()
        W.add_store_sums(host)
        st = eng.read_store()
        np.testing.assert_array_equal(st["expiry_ns"], host["expiry_ns"], err_msg=f"tick {rnd}")
        np.testing.assert_array_equal(st["subclients"], host["subclients"], err_msg=f"tick {rnd}")
        assert st["has"].tobytes() == gets.tobytes()
        rows = np.sort(rng.choice(N, 64, replace=False))  # the scattered-row read (server path)
        g2, e2 = eng.leases_rows(rows)
        np.testing.assert_array_equal(e2, exp[rows])
        assert g2.tobytes() == gets[rows].tobytes()


def test_config_limits_and_cold_fields_round_trip(eng):
    """Lease length and refresh interval are int32 seconds on the device (the hot 32-B
    config record and the cold record): values up to 2^31 - 1 round-trip through
    dm_read_config / dm_read_leases, 2^31 is DM_E_INVAL, and the safe capacity read
    back from the cold record is the configured one (or capacity / Count when unset)."""
    from doorman_amd._lib import DM_E_INVAL, DmError
    snap = W.make_snapshot([3, 2], np.ones(5), np.zeros(5), 1, NOW + W.NS, 1, 10.0)
    snap["lease_length_s"] = np.array([2 ** 31 - 1, 7], np.int64)
    snap["refresh_interval_s"] = np.array([2 ** 31 - 1, 3], np.int64)
    snap["safe_capacity"] = np.array([np.nan, 4.5])
    eng.load(snap)
    cfg = eng.config()
    assert cfg["lease_length_s"].tolist() == [2 ** 31 - 1, 7]
    assert cfg["refresh_interval_s"].tolist() == [2 ** 31 - 1, 3]
    eng.apportion(NOW, writeback=True)
    res = eng.resources()
    assert res["safe_capacity"][0] == 10.0 / 3 and res["safe_capacity"][1] == 4.5
    gets, exp = eng.leases()
    assert exp[:3].tolist() == [NOW + (2 ** 31 - 1) * W.NS] * 3 and exp[3:].tolist() == [NOW + 7 * W.NS] * 2
    bad = dict(snap)
    bad["lease_length_s"] = np.array([2 ** 31, 7], np.int64)
    with pytest.raises(DmError) as e:
        eng.load(bad)
    assert e.value.code == DM_E_INVAL


@pytest.mark.parametrize("expired", [0.0, 0.03])
@pytest.mark.parametrize("split", ["1", "0", "3"])
@pytest.mark.parametrize("cols", ["inplace", "alternate"])
def test_dense_subclients_state(monkeypatch, cols, split, expired):
    """A writeback tick marks a group-kernel resource dense when every live row is a
    follower with one subclient count (every other row is released then: its rows go
    into the resource's released-row mask); the next ticks skip its subclients
    column.  Releases and upserts (other subclient counts, explicit expiries, a
    released slot taken again) end the state until the next writeback tick, lapsed
    followers end it, wants refreshes keep it; every tick matches the oracle on a
    host copy, and dm_store_stats counts the dense resources.  split=1: after a
    writeback tick the workgroup bins (128x4, 128x8, 256x8, 512x8) run as
    k_block_dense + k_block_rest (stale hints queued); split=0 (DM_DENSE_SPLIT=0):
    the one-kernel form; split=3: only the 128-thread bins split.  expired > 0:
    loaded rows already past their expiry, released by the first tick (C2's shape),
    so most resources carry a mask from the start."""
    from doorman_amd.engine import Engine
    monkeypatch.setenv("DM_DENSE_SPLIT", split)  # read when the context is created
    eng = Engine(0)
    rng = np.random.default_rng(5150)
    sizes = np.array([12, 30, 60, 100, 200, 400, 900, 1000, 1500, 3000, 5, 0, 9000, 20, 700])
    snap = snapshot_with_sizes(rng, sizes, kinds=(1, 2, 3), expired_frac=expired, learning_frac=0.0,
                               parent_expired_frac=0.0)
    snap["lease_length_s"] = np.full(len(sizes), 20, np.int64)
    free = np.flatnonzero(rng.random(len(snap["wants"])) < expired)  # free slots too
    snap["expiry_ns"][free], snap["subclients"][free], snap["has"][free], snap["wants"][free] = W.RELEASED, 0, 0.0, 0.0
    W.add_store_sums(snap)
    group = (sizes >= 257) & (sizes <= 4096)  # the workgroup kernels keep the state
    eng.load(snap)
    assert eng.store_stats()["dense_resources"] == 0  # loaded rows carry explicit expiries
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    off = np.asarray(snap["seg_off"])
    N = len(host["wants"])
    for rnd, dt in enumerate([0, 5, 10, 15, 20, 25, 70]):
        now = NOW + dt * W.NS
        if rnd == 2:  # releases: those resources stop being dense
            rows = np.array([off[1] + 3, off[6] + 10, off[8] + 1])
            eng.release(rows)
            host["has"][rows], host["wants"][rows], host["subclients"][rows] = 0.0, 0.0, 0
            host["expiry_ns"][rows] = W.RELEASED
            W.add_store_sums(host)
        if rnd == 3:  # wants refreshes keep the state
            rows = np.sort(rng.choice(N, N // 10, replace=False))
            nw = rng.uniform(0.0, 2.0, len(rows))
            eng.update_wants(rows, nw)
            host["wants"][rows] = np.where(host["expiry_ns"][rows] == W.RELEASED, host["wants"][rows], nw)
            W.add_store_sums(host)
        if rnd == 4:  # upserts with another subclient count: explicit rows, non-uniform resources
            rows = np.array([off[2] + 5, off[7] + 2, off[9] + 7, off[1] + 3, off[6] + 10])
            ne = now + 100 * W.NS
            eng.upsert(rows, np.zeros(5), np.ones(5), np.full(5, 3, np.int64), np.full(5, ne))
            host["wants"][rows], host["has"][rows], host["subclients"][rows], host["expiry_ns"][rows] = 1.0, 0.0, 3, ne
            W.add_store_sums(host)
        eng.apportion(now, writeback=True, wb_columns=cols)
        gets, exp = eng.leases()
        ref = O.apportion(host, now)
        assert_leases_match(host, gets, exp, ref, f"tick {rnd}")
        live = ref["expiry_ns"] != W.RELEASED
        host["has"] = np.where(live, ref["gets"], 0.0)
        host["wants"] = np.where(live, host["wants"], 0.0)
        host["subclients"] = np.where(live, host["subclients"], 0)
        host["expiry_ns"] = ref["expiry_ns"].copy()
        W.add_store_sums(host)
        st = eng.read_store()
        np.testing.assert_array_equal(st["subclients"], host["subclients"], err_msg=f"tick {rnd}")
        np.testing.assert_array_equal(st["expiry_ns"], host["expiry_ns"], err_msg=f"tick {rnd}")
        # expected dense resources: 257-4096 rows, every live row with one subclient
        # count in 1..254 (released rows beside them), or no live row at all
        want = 0
        for r in np.flatnonzero(group):
            lv = host["expiry_ns"][off[r]:off[r + 1]] != W.RELEASED
            s = host["subclients"][off[r]:off[r + 1]][lv]
            want += int(not lv.any() or (s.min() == s.max() and 1 <= s[0] <= 254))
        assert eng.store_stats()["dense_resources"] == want, f"tick {rnd}"
    # every follower lapsed at the last tick: all released, the workgroup-bin resources stay dense
    assert eng.store_stats()["dense_resources"] == int(group.sum())
    eng.close()


def _writeback_and_check(eng, host, now, label):
    """One writeback tick against the oracle on the host copy, which then takes the tick's state."""
    eng.apportion(now, writeback=True)
    gets, exp = eng.leases()
    ref = O.apportion(host, now)
    assert_leases_match(host, gets, exp, ref, label)
    live = ref["expiry_ns"] != W.RELEASED
    host["has"] = np.where(live, ref["gets"], 0.0)
    host["wants"] = np.where(live, host["wants"], 0.0)
    host["subclients"] = np.where(live, host["subclients"], 0)
    host["expiry_ns"] = ref["expiry_ns"].copy()
    W.add_store_sums(host)


def test_dense_split_skips_the_rest_kernel_once_verified():
    """Within one row epoch (no call that writes rows since), a workgroup bin whose
    items were all counted dense after a writeback tick (k_count_undense) runs the
    dense kernel alone; a wants refresh (here a NaN wants, which ends a resource's
    dense state) starts a new epoch and the rest kernel runs again until the next
    check; followers that lapse together keep their resource dense (every row in its
    mask).  Every tick matches the oracle on a host copy."""
    from doorman_amd.engine import Engine
    eng = Engine(0)
    rng = np.random.default_rng(77)
    sizes = np.concatenate([rng.integers(257, 4097, 24), [5, 0, 40]])
    snap = snapshot_with_sizes(rng, sizes, kinds=(1, 2, 3), expired_frac=0.02, learning_frac=0.0,
                               parent_expired_frac=0.0)
    snap["lease_length_s"] = np.full(len(sizes), 20, np.int64)
    eng.load(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    off = np.asarray(snap["seg_off"])
    eng.set_profiling(True)

    def rest_launches():
        return sum(v[0] for k, v in eng.kernel_times().items() if k.endswith("_rest"))

    for t in range(4):
        eng.reset_kernel_times()
        _writeback_and_check(eng, host, NOW, f"tick {t}")
        if t == 3:  # tick 0 mixed + the check, tick 1 split with rest (record not read yet or read), then skipped
            assert rest_launches() == 0, eng.kernel_times()
            assert any(k.endswith("_dense") for k in eng.kernel_times())
    fs = [r for r in range(24) if host["kind"][r] == 3]
    assert fs, "no FairShare resource among the sampled kinds"
    row = int(off[fs[0]] + np.flatnonzero(host["expiry_ns"][off[fs[0]]:off[fs[0] + 1]] != W.RELEASED)[0])
    eng.update_wants(np.array([row]), np.array([np.nan]))
    host["wants"][row] = np.nan
    W.add_store_sums(host)
    eng.reset_kernel_times()
    _writeback_and_check(eng, host, NOW, "after the NaN refresh")
    kt = eng.kernel_times()  # a new epoch: every item decided by a kernel that reads the column
    assert rest_launches() >= 1 or any(k.startswith("block") and not k.endswith("_dense") for k in kt), kt
    for t in range(3):  # checked again in the new epoch (the NaN resource is not dense: the rest kernel stays)
        eng.reset_kernel_times()
        _writeback_and_check(eng, host, NOW, f"new epoch tick {t}")
    assert rest_launches() >= 1, eng.kernel_times()
    for t, dt in enumerate([5, 30, 31, 32]):  # the followers lapse at +20 s: all rows released, still dense
        _writeback_and_check(eng, host, NOW + dt * W.NS, f"lapse tick {t}")
    assert eng.store_stats()["dense_resources"] == 24
    eng.close()


def _c4_store(rng, R, n, learning_frac=0.05, short_frac=0.1):
    """configs[4]'s store shape at test size: FS/PS mixed, 5% learning resources, 2%
    free slots, loaded rows with explicit expiries (some already past), and a tenth
    of the resources with a 4-s lease (shorter than the 5-s round: their leases lapse
    between ticks, so every round's Clean releases rows)."""
    snap = W.uniform(R, n, kind="mixed", seed=int(rng.integers(1 << 30)))
    snap["learning_end_ns"] = np.where(rng.random(R) < learning_frac, NOW + 3600 * W.NS, W.INT64_MIN).astype(np.int64)
    snap["lease_length_s"] = np.where(rng.random(R) < short_frac, 4, 300).astype(np.int64)
    N = len(snap["wants"])
    free = rng.random(N) < 0.02
    snap["wants"][free] = 0.0
    snap["has"][free] = 0.0
    snap["subclients"] = np.where(free, 0, 1).astype(np.int64)
    snap["expiry_ns"] = np.where(free, W.RELEASED, NOW + rng.integers(-20, 3600, N) * W.NS).astype(np.int64)
    return W.add_store_sums(snap)


def _c4_round(rng, host, now):
    """One round's updates as bench.streaming_step makes them: 10% wants refresh as a
    row mask + packed values, 1% departures, arrivals into free rows."""
    N = len(host["wants"])
    alive = np.flatnonzero(host["expiry_ns"] != W.RELEASED)
    upd = np.sort(rng.choice(alive, len(alive) // 10, replace=False))
    w = rng.uniform(0.5, 1.5, len(upd))
    rest = np.setdiff1d(alive, upd)
    gone = np.sort(rng.choice(rest, max(1, len(alive) // 100), replace=False))
    pool = np.setdiff1d(np.flatnonzero(host["expiry_ns"] == W.RELEASED), gone)
    new = np.sort(rng.choice(pool, min(len(pool), len(gone)), replace=False))
    k = len(new)
    return (W.rows_to_mask(upd, N), w, gone, new, np.zeros(k), rng.uniform(0.5, 1.5, k), np.ones(k, np.int64),
            np.full(k, now + 3600 * W.NS, np.int64), upd)


def _apply_host(host, upd, w, gone, new, nh, nw, ns, ne):
    """The same round on the host copy: Assign of the new wants (store.go:153-167),
    Release (store.go:142-151), Assign of the arrivals."""
    host["wants"][upd] = w
    for k, v in (("wants", 0.0), ("has", 0.0), ("subclients", 0), ("expiry_ns", W.RELEASED)):
        host[k][gone] = v
    host["wants"][new], host["has"][new], host["subclients"][new], host["expiry_ns"][new] = nw, nh, ns, ne
    W.add_store_sums(host)


def _writeback_host(host, ref):
    live = ref["expiry_ns"] != W.RELEASED
    host["has"] = np.where(live, ref["gets"], 0.0)
    host["wants"] = np.where(live, host["wants"], 0.0)
    host["subclients"] = np.where(live, host["subclients"], 0)
    host["expiry_ns"] = ref["expiry_ns"].copy()


@pytest.mark.parametrize("cols,narrow,asynchronous", [("inplace", False, False), ("alternate", False, False),
                                                      ("inplace", True, False), ("alternate", True, True)])
def test_c4_loop_store_apply_matches_oracle(eng, cols, narrow, asynchronous):
    """configs[4]'s own loop under the oracle.  Every 5-s round the bench's
    update call -- dm_store_apply with the wants refresh as a row mask, departures and
    arrivals -- then a writeback tick; 5% learning resources, leases that lapse
    between rounds (4-s lease resources, loaded rows whose explicit expiry passes).
    A host copy takes the same updates and each tick's writeback; the oracle decides
    every round (store.go:142-181, resource.go:108-111) from exact sums while the
    device uses its running sums.  narrow: the arrivals as bench.py sends them -- row,
    wants, int32 subclients, has and expiry implied (0 and now + the resource's lease
    length, the Assign of a new client).  asynchronous: each round's batch through
    dm_store_apply_async and the tick enqueued behind it, as bench.py's C4 step (the
    store's sums read back every other round; test_c4_rounds_async_back_to_back below
    keeps several rounds in flight)."""
    rng = np.random.default_rng(404)
    snap = _c4_store(rng, 2000, 300)
    eng.load(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    now = NOW
    released_by_clean = 0
    for rnd in range(6):
        now += 5 * W.NS
        mask, w, gone, new, nh, nw, ns, ne, upd = _c4_round(rng, host, now)
        if narrow:
            so = snap["seg_off"]
            ne = now + snap["lease_length_s"][np.searchsorted(so, new, side="right") - 1] * W.NS
            eng.apply(mask, w, gone, (new, None, nw, ns.astype(np.int32), None), now_ns=now, asynchronous=asynchronous)
        else:
            eng.apply(mask, w, gone, (new, nh, nw, ns, ne), asynchronous=asynchronous)
        _apply_host(host, upd, w, gone, new, nh, nw, ns, ne)
        if not asynchronous or rnd % 2 == 0:
            res = eng.resources(safe=False)
            np.testing.assert_array_equal(res["count"], host["agg_count"])  # the running Count, exact
            assert float_close(res["sum_wants"], host["agg_sum_wants"], np.maximum(snap["capacity"], 1.0)).all()
        eng.apportion(now, writeback=True, wb_columns=cols, asynchronous=asynchronous)
        gets, exp = eng.leases()
        ref = O.apportion(host, now)
        assert_leases_match(host, gets, exp, ref, f"C4 loop round {rnd}")
        released_by_clean += int(((host["expiry_ns"] != W.RELEASED) & (ref["expiry_ns"] == W.RELEASED)).sum())
        _writeback_host(host, ref)
    assert released_by_clean > 0  # Clean released leases during the loop
    if asynchronous:
        eng.apply_wait()
    st = eng.read_store()
    for k in ("subclients", "expiry_ns"):
        np.testing.assert_array_equal(st[k], host[k])


@pytest.mark.parametrize("n,R,fs_only", [(300, 2000, False), (800, 1000, False), (1500, 500, False),
                                         (3000, 300, False), (800, 5000, True)],
                         ids=["bin3_128x4", "bin4_128x8", "bin5_256x8", "bin6", "bin4_wave_64x16"])
def test_dense_state_survives_releases_and_arrivals(eng, n, R, fs_only):
    """configs[4]'s rounds keep the workgroup bins' resources dense.  A
    release marks its row in the released-row mask and an arrival (the resource's count,
    the Assign's expiry) goes into the arrival mask instead of ending the dense state
    (dm_device.h DenseUpd), for every bin shape (the nibble-packed 128 x 4, 128 x 8,
    256 x 8, bin 6, and bin 4's one-wave 64 x 16 shape of a FairShare store in stream
    parts).  Rounds as the bench's (narrow arrivals, row-mask wants refresh), a tenth of
    the resources on a 4-s lease so their followers lapse while arrivals made at the
    round's time outlive them (the column path).  Each tick against the oracle; the dense
    share at tick time (dm_store_stats) after each round's updates; the store read back
    equal to the host's copy at the end."""
    rng = np.random.default_rng(505 + n)
    snap = _c4_store(rng, R, n)
    if fs_only:
        snap["kind"] = np.full(R, W.FAIR_SHARE, np.int32)
    eng.load(snap)
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    now = NOW
    so = snap["seg_off"]
    for t in range(2):  # writeback ticks: every resource dense (released rows in its mask)
        eng.apportion(now, writeback=True)
        ref = O.apportion(host, now)
        _writeback_host(host, ref)
        W.add_store_sums(host)
    shares = []
    for rnd in range(5):
        now += 5 * W.NS
        mask, w, gone, new, nh, nw, ns, ne, upd = _c4_round(rng, host, now)
        ne = now + snap["lease_length_s"][np.searchsorted(so, new, side="right") - 1] * W.NS
        eng.apply(mask, w, gone, (new, None, nw, ns.astype(np.int32), None), now_ns=now)
        _apply_host(host, upd, w, gone, new, nh, nw, ns, ne)
        st = eng.store_stats()
        shares.append(st["dense_leases"] / len(host["wants"]))
        eng.apportion(now, writeback=True)
        gets, exp = eng.leases()
        ref = O.apportion(host, now)
        assert_leases_match(host, gets, exp, ref, f"round {rnd}")
        _writeback_host(host, ref)
        W.add_store_sums(host)
        res = eng.resources(safe=False)
        np.testing.assert_array_equal(res["count"], host["agg_count"])
    # the 4-s resources lapse every round; the rest keep their dense state through the updates
    assert min(shares) >= 0.8, shares
    st = eng.read_store()
    for k in ("subclients", "expiry_ns"):
        np.testing.assert_array_equal(st[k], host[k], err_msg=k)
    assert float_close(st["has"], host["has"], row_capacity(host)).all()
    if fs_only:
        assert eng.plan_info()["bin_shapes"] & 2  # bin 4 ran on one wave per resource


def test_c4_full_size_properties_after_bench_rounds(eng):
    """configs[4] at full per-GPU size (125M leases, bench.make_workload("c4")):
    three of the bench's own rounds (bench.streaming_step: dm_store_apply_async +
    writeback tick, enqueued back to back), then size-independent properties over every resource: the running Count
    equals the live rows (bit-exact; every client has one subclient) and the running
    SumHas equals the sum of the live leases' gets within 1e-9 * capacity."""
    import bench
    snap = bench.make_workload("c4", 0)
    eng.load(snap)
    step = bench.streaming_step(eng, snap, 0, 3)
    for _ in range(3):
        step()
    eng.sync()
    step.finish()  # the rounds' asynchronous batches retired: none rejected
    gets, exp = eng.leases()
    res = eng.resources(safe=False)
    so = snap["seg_off"]
    live = exp != W.RELEASED
    np.testing.assert_array_equal(res["count"], np.add.reduceat(live.astype(np.int64), so[:-1]))
    per_res = np.add.reduceat(np.where(live, gets, 0.0), so[:-1])
    np.testing.assert_allclose(res["sum_has"], per_res, rtol=0, atol=1e-9 * 1000.0)
    assert live.sum() > 0.97 * len(live)
    del snap, gets, exp, live


def test_configs0_through_the_hip_path(eng):
    """BASELINE configs[0] (1 resource x 1,000 clients, ProportionalShare,
    algorithm.go:213-293) through dm_apportion: every lease against the oracle's
    literal per-request Decide (one private store copy per client) and its closed
    form; then three writeback ticks against the oracle replaying them."""
    snap = W.c0()
    eng.load(snap)
    eng.apportion(NOW)
    gets, exp = eng.leases()
    for mode in ("literal", "closed"):
        ref = O.apportion(snap, NOW, mode=mode)
        assert_leases_match(snap, gets, exp, ref, f"configs[0] vs oracle {mode}")
        assert_resources_match(snap, eng.resources(), ref, f"configs[0] {mode}")
    host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
    for t in range(3):
        now = NOW + t * W.NS
        eng.apportion(now, writeback=True)
        gets, exp = eng.leases()
        ref = O.apportion(host, now, mode="literal")
        assert_leases_match(host, gets, exp, ref, f"configs[0] writeback tick {t}")
        _writeback_host(host, ref)
        W.add_store_sums(host)


def test_dense_split_queues_undecided_items():
    """The split form with items the dense kernel cannot decide (no dense hint: a
    released row or mixed subclient counts) queued for k_block_rest every tick:
    resources in all four workgroup bins, FairShare with mixed counts (handed to
    k_general), ProportionalShare, Static; writeback ticks back to back (no store
    update between, so the split form runs), every tick against the oracle on the
    device store as it stood, and gets bit-identical to the one-kernel form
    (DM_DENSE_SPLIT=0)."""
    import os
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(8088)
    sizes = np.concatenate([rng.integers(257, 513, 12), rng.integers(513, 1025, 12), rng.integers(1025, 2049, 8),
                            rng.integers(2049, 4097, 6)])
    R, N = len(sizes), int(sizes.sum())
    snap = snapshot_with_sizes(rng, sizes, kinds=(1, 2, 3), expired_frac=0.0, learning_frac=0.0,
                               parent_expired_frac=0.0)
    snap["lease_length_s"] = np.full(R, 300, np.int64)
    snap["expiry_ns"] = np.full(N, NOW + 600 * W.NS, np.int64)
    off = np.asarray(snap["seg_off"])
    sub = np.ones(N, np.int64)
    for r in range(0, R, 5):  # a released row: never dense, streamed every tick
        snap["expiry_ns"][off[r] + 7] = W.RELEASED
    for r in range(2, R, 7):  # mixed subclient counts: PS streamed, FS to k_general
        sub[off[r]:off[r + 1]] = rng.integers(1, 4, sizes[r])
    snap["subclients"] = sub
    snap.pop("agg_count", None), snap.pop("agg_sum_has", None), snap.pop("agg_sum_wants", None)
    old = os.environ.get("DM_DENSE_SPLIT")
    os.environ["DM_DENSE_SPLIT"] = "1"
    a = Engine(0)
    os.environ["DM_DENSE_SPLIT"] = "0"
    b = Engine(0)
    if old is None:
        os.environ.pop("DM_DENSE_SPLIT")
    else:
        os.environ["DM_DENSE_SPLIT"] = old
    try:
        a.load(snap)
        b.load(snap)
        a.set_profiling(True)
        for i in range(5):
            now = NOW + i * 5 * W.NS
            st, res = a.read_store(), a.resources(safe=False)
            cur = dict(snap)
            cur.update(has=st["has"], wants=st["wants"], subclients=st["subclients"], expiry_ns=st["expiry_ns"],
                       agg_count=res["count"], agg_sum_has=res["sum_has"], agg_sum_wants=res["sum_wants"])
            ref = O.apportion(cur, now)
            a.apportion(now, writeback=True)
            b.apportion(now, writeback=True)
            ga, gb = a.read_store()["has"], b.read_store()["has"]
            live = ref["expiry_ns"] != W.RELEASED
            assert float_close(np.where(live, ga, 0.0), np.where(live, ref["gets"], 0.0), row_capacity(cur)).all(), \
                f"tick {i}"
            assert ga.tobytes() == gb.tobytes(), f"tick {i}: dense form differs from the one-kernel form"
        a.sync()
        kt = a.kernel_times()
        assert any(k.endswith("_dense") and v[0] > 0 for k, v in kt.items()), kt
    finally:
        a.close()
        b.close()


def test_arrivals_without_expiry_need_a_clock():
    """arrivals whose expiry is implied (now + the resource's lease length)
    need the caller's now: Engine.apply refuses to default it, and dm_store_apply
    rejects upsert_now_ns <= 0 with DM_E_INVAL before anything is written."""
    import ctypes
    from doorman_amd import _lib
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(5)
    snap = snapshot_with_sizes(rng, np.array([300, 20, 5000], np.int64), expired_frac=0.0)
    free = np.array([3, 310, 400], np.int64)
    for k, v in (("wants", 0.0), ("has", 0.0), ("subclients", 0), ("expiry_ns", W.RELEASED)):
        snap[k][free] = v
    W.add_store_sums(snap)
    with Engine(0) as e:
        e.load(snap)
        before = e.read_store()
        arrivals = (free, None, np.ones(3), np.ones(3, np.int32), None)
        with pytest.raises(ValueError):
            e.apply(upsert=arrivals)
        b = _lib.StoreBatch()
        rows, w, s32 = free.copy(), np.ones(3), np.ones(3, np.int32)
        b.upsert_n, b.upsert_rows, b.upsert_wants = 3, rows.ctypes.data, w.ctypes.data
        b.upsert_subclients32 = s32.ctypes.data
        b.upsert_now_ns = 0
        assert e._L.dm_store_apply(e._ctx, ctypes.byref(b)) == _lib.DM_E_INVAL
        after = e.read_store()
        for k in before:
            assert before[k].tobytes() == after[k].tobytes(), k
        e.apply(upsert=arrivals, now_ns=W.NOW_NS)  # with the clock: the leases expire now + lease length
        got = e.read_store()
        np.testing.assert_array_equal(got["expiry_ns"][free],
                                      W.NOW_NS + np.repeat(snap["lease_length_s"], np.diff(snap["seg_off"]))[free] * W.NS)
