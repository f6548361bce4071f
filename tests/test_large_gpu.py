"""Large resources (> 4096 rows): the five-launch chain (every chunk re-derives the
resource's totals from the previous launch's partials), the one-launch path
(DM_LARGE_FUSED, dm_large.hip: rows resident in VGPRs, totals exchanged in-launch) and
the persistent task-queue path (DM_LARGE_FLOW, dm_flow.hip: the chain's phases as
listed tasks of one launch, totals reduced once per resource) against each other and
against the oracle (SURVEY.md §8c bar, with the observed error reported).  Each path
is deterministic; they differ only in the rounding of their per-resource sums
(different chunking and reduction trees)."""
import os

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import (assert_leases_match, assert_resources_match, binned_sizes, float_close, row_capacity,
                         snapshot_with_sizes)

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS


def _engine(G=None, fused=False, path=None, env=None):
    from doorman_amd.engine import Engine
    env = dict(env or {})
    if G is not None:
        env["DM_FUSED_G"] = str(G)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e = Engine(0)
        e.set_large_path(fused=fused, path=path)
        return e
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def pair():
    fused, chain = _engine(fused=True), _engine()
    yield fused, chain
    fused.close()
    chain.close()


@pytest.fixture(scope="module")
def flow():
    e = _engine(path="flow")
    yield e
    e.close()


def _tick(eng, snap, **kw):
    eng.load(snap)
    eng.apportion(NOW, **kw)
    gets, exp = eng.leases()
    return gets, exp, eng.resources()


def _same(snap, a, b, label):
    """Integers bit-exact, floats within the survey's bar (the two paths' sums round
    differently)."""
    ga, ea, ra = a
    gb, eb, rb = b
    assert ea.tobytes() == eb.tobytes(), f"{label}: expiry differs"
    np.testing.assert_array_equal(ra["count"], rb["count"], err_msg=f"{label}: count")
    ok = float_close(ga, gb, row_capacity(snap))
    if not ok.all():
        bad = np.flatnonzero(~ok)[:8]
        raise AssertionError(f"{label}: gets differ at rows {bad.tolist()}: {ga[bad].tolist()} vs {gb[bad].tolist()}")
    cap = np.maximum(np.abs(np.asarray(snap["capacity"], dtype=np.float64)), 1.0)
    for k in ("sum_wants", "safe_capacity"):
        assert float_close(ra[k], rb[k], cap).all(), f"{label}: {k} differs"


def _deterministic(eng, snap, first, label, **kw):
    again = _tick(eng, snap, **kw)
    for x, y in zip(first[:2], again[:2]):
        assert x.tobytes() == y.tobytes(), f"{label}: not deterministic"


def large_sizes(rng, n=12):
    """Large resources around the fused chunk edges (256 x 8 = 2048 and 512 x 8 = 4096
    rows) plus some much larger ones, mixed with every other bin."""
    big = [4097, 6143, 6144, 8192, 8193, 12288, 16385, 40000, 65536, 100001]
    sizes = list(binned_sizes(rng, per_bin=2)) + big + list(rng.integers(4097, 30000, n))
    rng.shuffle(sizes)
    return np.asarray(sizes, dtype=np.int64)


def max_err(snap, gets, ref):
    """max |got - ref| / max(|ref|, C_r / n_r) over live rows: a floor of one client's
    equal share instead of the survey's C_r, so a bias on the large
    path cannot hide under the capacity floor."""
    so = snap["seg_off"]
    n_of_row = np.maximum(np.repeat(np.diff(so), np.diff(so)), 1)
    floor = np.abs(row_capacity(snap)) / n_of_row
    live = ref["expiry_ns"] != W.RELEASED
    r = ref["gets"][live]
    g = gets[live]
    fin = np.isfinite(r) & np.isfinite(g)
    assert (g[~fin].tobytes() == r[~fin].tobytes()) or np.array_equal(np.isnan(g[~fin]), np.isnan(r[~fin]))
    denom = np.maximum(np.abs(r[fin]), floor[live][fin])
    with np.errstate(invalid="ignore", divide="ignore"):
        e = np.where(denom > 0, np.abs(g[fin] - r[fin]) / denom, np.abs(g[fin] - r[fin]))
    return float(e.max()) if e.size else 0.0


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("variant", ["uniform", "hetero", "edge", "recompute", "no_expiry", "learning"])
def test_fused_matches_chain(pair, seed, variant):
    fused, chain = pair
    rng = np.random.default_rng(9000 + seed)
    snap = snapshot_with_sizes(rng, large_sizes(rng), hetero=variant == "hetero", edge=variant == "edge",
                               expired_frac=0.0 if variant == "no_expiry" else 0.05,
                               learning_frac=0.5 if variant == "learning" else 0.1)
    rec = variant == "recompute"
    if rec:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            snap.pop(k)
    a = _tick(fused, snap, recompute=rec)
    assert fused.plan_info()["large_fused"] == 1
    assert chain.plan_info()["large_fused"] == 0
    b = _tick(chain, snap, recompute=rec)
    _same(snap, a, b, f"seed={seed} {variant}")
    _deterministic(fused, snap, a, f"seed={seed} {variant}", recompute=rec)


@pytest.mark.parametrize("path", ["chain", "fused256", "fused512"])
@pytest.mark.parametrize("kinds", [(2,), (3,), (0, 1, 2, 3)])
def test_large_against_oracle(path, kinds):
    """Both paths (and both chunk shapes of the one-launch path) against the oracle;
    the observed error is reported beside the survey's 1e-9 bar and must meet it
    with the per-client floor too."""
    rng = np.random.default_rng(len(path) + len(kinds))
    G = int(path[5:]) if path != "chain" else None
    eng = _engine(G, fused=G is not None)
    try:
        sizes = np.asarray([4097, 8192, 8193, 20000, 33333, 65537], dtype=np.int64)
        snap = snapshot_with_sizes(rng, sizes, kinds=kinds)
        gets, exp, res = _tick(eng, snap)
        info = eng.plan_info()
        if G is not None:
            assert info["large_fused"] == 1 and info["fused_chunks"] == int(np.sum(-(-sizes // (G * 8))))
        else:
            assert info["large_fused"] == 0 and info["large_chunks"] == int(np.sum(-(-sizes // 2048)))
    finally:
        eng.close()
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, path)
    assert_resources_match(snap, res, ref, path)
    e = max_err(snap, gets, ref)
    print(f"\n{path} kinds={kinds}: max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9


def test_fused_writeback_sequence_matches_chain(pair):
    """Several writeback ticks (the hand-off state is reused launch after launch:
    counters reset by their last arriver, flags tagged with the launch epoch),
    synchronous and deferred-join asynchronous, against the chain."""
    fused, chain = pair
    rng = np.random.default_rng(77)
    snap = snapshot_with_sizes(rng, large_sizes(rng, n=20), kinds=(2, 3), expired_frac=0.02)
    fused.load(snap)
    chain.load(snap)
    for i in range(6):
        now = NOW + i * 5 * W.NS
        for e in (fused, chain):
            e.apportion(now, writeback=True, asynchronous=i % 2 == 1, defer_join=i % 2 == 1)
            e.sync()
        a = (*fused.leases(), fused.resources())
        b = (*chain.leases(), chain.resources())
        _same(snap, a, b, f"tick {i}")


@pytest.mark.parametrize("which", ["chain", "fused"])
def test_large_resources_at_c2(pair, which):
    """configs[2]'s large resources (up to 1M rows: 489 chunks of 2048) through both
    paths (the one-launch path fits the residency bound here), sampled against the
    oracle with the error reported."""
    eng = pair[0] if which == "fused" else pair[1]
    snap = W.c2()
    eng.load(snap)
    info = eng.plan_info()
    print(f"\nC2 plan: {info}")
    if which == "fused":
        assert info["large_fused"] == 1 and 2 * info["fused_max_chunks"] <= info["fused_capacity"]
    eng.apportion(NOW)
    gets, exp = eng.leases()
    so = snap["seg_off"]
    sample = np.asarray([0, 1, 2, 3, 10, 50, 121, 200, 243], dtype=np.int64)  # the largest resources
    sub = W.subset(snap, sample)
    ref = O.apportion(sub, NOW)
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in sample])
    assert_leases_match(sub, gets[rows], exp[rows], ref, f"C2 large {which}")
    e = max_err(sub, gets[rows], ref)
    print(f"C2 large resources ({which}): max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9


def test_fused_wait_that_gives_up_loses_the_store_until_reload():
    """a fused-path wait that gives up (forced here with a zero spin bound,
    DM_FUSED_SPIN_LIMIT) fails the tick with DM_E_HIP, and the chunk stops before
    any further store write.  Chunks that did get their totals may have written
    their rows, so after a failed writeback tick every call that needs the store
    reports DM_E_STATE until the store is loaded again; the reloaded store then
    ticks exactly as the chain does.  A failed tick without writeback keeps the
    store."""
    from doorman_amd._lib import DM_E_HIP, DM_E_STATE
    from doorman_amd._lib import DmError as DoormanError
    rng = np.random.default_rng(77)
    snap = snapshot_with_sizes(rng, np.array([60000, 70000, 50000, 45000], dtype=np.int64), hetero=False)
    os.environ["DM_FUSED_SPIN_LIMIT"] = "0"
    try:
        eng = _engine(fused=True)
    finally:
        os.environ.pop("DM_FUSED_SPIN_LIMIT")
    chain = _engine()
    try:
        eng.load(snap)
        before = eng.read_store()
        try:
            eng.apportion(NOW)  # no writeback: the store must survive a failure
            failed = False
        except DoormanError as e:
            assert e.code == DM_E_HIP
            failed = True
        after = eng.read_store()
        for k in before:
            assert before[k].tobytes() == after[k].tobytes(), k
        assert failed, "a zero spin bound must make some chunk's wait give up"
        if failed:
            with pytest.raises(DoormanError) as e:
                eng.apportion(NOW, writeback=True)
            assert e.value.code == DM_E_HIP
            for call in (lambda: eng.apportion(NOW), lambda: eng.read_store(), lambda: eng.leases()):
                with pytest.raises(DoormanError) as e:
                    call()
                assert e.value.code == DM_E_STATE
        eng.set_large_path(fused=False)
        a = _tick(eng, snap, writeback=True)
        b = _tick(chain, snap, writeback=True)
        for x, y in zip(a[:2], b[:2]):
            assert x.tobytes() == y.tobytes()
    finally:
        eng.close()
        chain.close()


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("variant", ["uniform", "hetero", "edge", "recompute", "no_expiry", "learning"])
def test_flow_matches_chain(pair, flow, seed, variant):
    """The persistent path against the chain on the same snapshots as the fused path
    (heterogeneous FairShare resources go to k_general either way)."""
    chain = pair[1]
    rng = np.random.default_rng(9000 + seed)
    snap = snapshot_with_sizes(rng, large_sizes(rng), hetero=variant == "hetero", edge=variant == "edge",
                               expired_frac=0.0 if variant == "no_expiry" else 0.05,
                               learning_frac=0.5 if variant == "learning" else 0.1)
    rec = variant == "recompute"
    if rec:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            snap.pop(k)
    a = _tick(flow, snap, recompute=rec)
    assert flow.plan_info()["large_flow"] == 1
    b = _tick(chain, snap, recompute=rec)
    _same(snap, a, b, f"seed={seed} {variant}")
    _deterministic(flow, snap, a, f"seed={seed} {variant}", recompute=rec)


@pytest.mark.parametrize("grid", ["1", "3", "default"])
@pytest.mark.parametrize("kinds", [(2,), (3,), (0, 1, 2, 3)])
def test_flow_against_oracle(grid, kinds):
    """The persistent path against the oracle, also drained by ONE workgroup and by
    three (the task list alone orders the phases: no co-residency is assumed)."""
    rng = np.random.default_rng(17 + len(kinds))
    eng = _engine(path="flow", env={} if grid == "default" else {"DM_FLOW_GRID": grid})
    try:
        sizes = np.asarray([4097, 8192, 8193, 20000, 33333, 65537, 5000, 250000], dtype=np.int64)
        snap = snapshot_with_sizes(rng, sizes, kinds=kinds, expired_frac=0.05)
        gets, exp, res = _tick(eng, snap)
        info = eng.plan_info()
        assert info["large_flow"] == 1 and info["large_chunks"] == int(np.sum(-(-sizes // 2048)))
        if grid != "default":
            assert info["flow_grid"] == int(grid)
        # pass A per chunk, round 1 per bundle of 8 chunks, round 2 and the map per chunk
        nch = -(-sizes // 2048)
        assert info["flow_tasks"] == int(3 * nch.sum() + np.sum(-(-nch // 8)))
    finally:
        eng.close()
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, f"flow grid={grid}")
    assert_resources_match(snap, res, ref, f"flow grid={grid}")
    e = max_err(snap, gets, ref)
    print(f"\nflow grid={grid} kinds={kinds}: max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9


def test_flow_writeback_sequence_matches_chain(pair, flow):
    """Writeback ticks with rows lapsing between them (round 1 recomputed from the rows
    where Clean releases subclients), synchronous and deferred-join asynchronous,
    against the chain: the ticket counters, arrive counters and epoch-tagged flags are
    reused launch after launch."""
    chain = pair[1]
    rng = np.random.default_rng(78)
    snap = snapshot_with_sizes(rng, large_sizes(rng, n=20), kinds=(0, 1, 2, 3), expired_frac=0.02)
    # explicit expiries from 10 s before the first tick (its Clean releases rows of
    # most resources: round 1 recomputed) and lease lengths of 3-20 s (later ticks
    # see whole resources lapse)
    live = snap["expiry_ns"] != W.RELEASED
    snap["expiry_ns"] = np.where(live, NOW + rng.integers(-10, 30, live.size) * W.NS, snap["expiry_ns"])
    snap["lease_length_s"] = rng.integers(3, 21, len(snap["lease_length_s"])).astype(np.int64)
    flow.load(snap)
    chain.load(snap)
    for i in range(6):
        now = NOW + i * 5 * W.NS
        for e in (flow, chain):
            e.apportion(now, writeback=True, asynchronous=i % 2 == 1, defer_join=i % 2 == 1)
            e.sync()
        a = (*flow.leases(), flow.resources())
        b = (*chain.leases(), chain.resources())
        _same(snap, a, b, f"tick {i}")


def test_flow_large_resources_at_c2(flow):
    """configs[2]'s large resources (up to 1M rows) through the persistent path,
    sampled against the oracle with the error reported."""
    snap = W.c2()
    flow.load(snap)
    info = flow.plan_info()
    assert info["large_flow"] == 1
    flow.apportion(NOW)
    gets, exp = flow.leases()
    so = snap["seg_off"]
    sample = np.asarray([0, 1, 2, 3, 10, 50, 121, 200, 243], dtype=np.int64)
    sub = W.subset(snap, sample)
    ref = O.apportion(sub, NOW)
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in sample])
    assert_leases_match(sub, gets[rows], exp[rows], ref, "C2 large flow")
    e = max_err(sub, gets[rows], ref)
    print(f"C2 large resources (flow): max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9


def test_flow_wait_that_gives_up_fails_the_tick():
    """A persistent-path wait that gives up (a zero spin bound) fails the tick with
    DM_E_HIP and, after a writeback tick, loses the store until it is reloaded (as the
    fused path); the reloaded store then ticks as the chain."""
    from doorman_amd._lib import DM_E_HIP, DM_E_STATE
    from doorman_amd._lib import DmError as DoormanError
    rng = np.random.default_rng(79)
    snap = snapshot_with_sizes(rng, np.array([60000, 70000, 50000, 45000], dtype=np.int64), hetero=False)
    eng = _engine(path="flow", env={"DM_FUSED_SPIN_LIMIT": "0"})
    chain = _engine()
    try:
        eng.load(snap)
        before = eng.read_store()
        failed = False
        try:
            eng.apportion(NOW)
        except DoormanError as e:
            assert e.code == DM_E_HIP
            failed = True
        after = eng.read_store()
        for k in before:
            assert before[k].tobytes() == after[k].tobytes(), k
        if failed:
            try:
                eng.apportion(NOW, writeback=True)
                lost = False
            except DoormanError as e:
                assert e.code == DM_E_HIP
                lost = True
            if lost:
                with pytest.raises(DoormanError) as e:
                    eng.read_store()
                assert e.value.code == DM_E_STATE
        eng.set_large_path(path="chain")
        a = _tick(eng, snap, writeback=True)
        b = _tick(chain, snap, writeback=True)
        for x, y in zip(a[:2], b[:2]):
            assert x.tobytes() == y.tobytes()
    finally:
        eng.close()
        chain.close()


def _store_as_snapshot(snap, eng):
    """The device store as it now stands, as an oracle snapshot (running sums included)."""
    st, res = eng.read_store(), eng.resources(safe=False)
    s = dict(snap)
    s.update(has=st["has"], wants=st["wants"], subclients=st["subclients"], expiry_ns=st["expiry_ns"],
             agg_count=res["count"], agg_sum_has=res["sum_has"], agg_sum_wants=res["sum_wants"])
    return s


def test_large_writeback_ticks_against_oracle():
    """Writeback ticks on large FairShare / ProportionalShare resources (the chain's
    speculative round 1 and the per-resource totals it leaves in SegTot reused tick
    after tick), each checked against the oracle on the device store as it stood
    before it.  Between ticks the wants change by nothing, by a little and by a lot,
    one resource loses its wantExtra clients entirely (T not finite), and one tick
    follows releases; one follows a non-writeback tick far in the future (every row
    lapsed in that tick's view, none in the store's).  Then arrivals with explicit expiries, some already past (Clean
    releases part of a resource: pass B recomputes round 1), and a tick after every
    follower's lease has lapsed (Clean releases all of them: pass A's speculative
    round 1 is still exact, so the chain runs without pass B)."""
    rng = np.random.default_rng(4242)
    sizes = np.asarray([4097, 6000, 8192, 20000, 65537, 150000], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=(3, 3, 3, 2), expired_frac=0.0, learning_frac=0.0)
    snap["expiry_ns"] = np.full(len(snap["wants"]), NOW + 3600 * W.NS, np.int64)
    so = snap["seg_off"]
    N = len(snap["wants"])
    eng = _engine()
    try:
        eng.load(snap)
        base = np.asarray(snap["wants"], dtype=np.float64).copy()
        plan = ["same", "same", "small", "same", "large", "peek", "same", "zero", "same", "release", "same", "arrive",
                "same", "lapse", "same"]
        worst = 0.0
        now = NOW
        for i, step in enumerate(plan):
            now += (1000 if step == "lapse" else 5) * W.NS  # leases are 1..600 s
            if step == "arrive":  # explicit expiries, half of them already past at this tick
                rows = rng.choice(N, 400, replace=False).astype(np.int64)
                st = eng.read_store()
                exp = np.where(rng.random(400) < 0.5, now - W.NS, now + 30 * W.NS).astype(np.int64)
                eng.upsert(rows, st["has"][rows], rng.uniform(0.0, 50.0, 400), np.ones(400, np.int64), exp)
            elif step == "peek":  # (the store's running sums read before it: resources() reads the last tick's)
                pre = _store_as_snapshot(snap, eng)
                eng.apportion(now + 10_000 * W.NS, writeback=False)
            elif step == "small":
                w = base * (1.0 + 1e-7 * rng.standard_normal(N))
                eng.update_wants(np.arange(N, dtype=np.int64), w)
            elif step == "large":
                w = base * rng.uniform(0.5, 2.0, N)
                eng.update_wants(np.arange(N, dtype=np.int64), w)
            elif step == "zero":  # resource 1 wants nothing: no wantExtra clients, T not finite
                rows = np.arange(so[1], so[2], dtype=np.int64)
                eng.update_wants(rows, np.zeros(len(rows)))
            elif step == "release":
                eng.release(rng.choice(N, 500, replace=False).astype(np.int64))
            cur = pre if step == "peek" else _store_as_snapshot(snap, eng)
            ref = O.apportion(cur, now)
            eng.apportion(now, writeback=True)
            st = eng.read_store()
            live = ref["expiry_ns"] != W.RELEASED
            gets = np.where(live, st["has"], 0.0)
            assert float_close(gets, np.where(live, ref["gets"], 0.0), row_capacity(cur)).all(), f"tick {i} ({step})"
            worst = max(worst, max_err(cur, gets, ref))
        print(f"\nlarge writeback ticks: max |got-ref|/max(|ref|, C_r/n_r) over {len(plan)} ticks = {worst:.3e}")
        assert worst <= 1e-9
    finally:
        eng.close()
