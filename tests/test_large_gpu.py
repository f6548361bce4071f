"""Large resources (> 4096 rows): the chunked chain (2048-row chunks; every chunk
re-derives the resource's totals from the previous launch's partials) against the
oracle (SURVEY.md §8c bar, with the observed error reported), its determinism, and
its writeback ticks tick after tick (the speculative round 1, the per-resource
totals it leaves, the subclients-free pass A of the steady state).  The one-launch
and persistent-queue forms of rounds 2-3 were retired in round 4."""
import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import (assert_leases_match, assert_resources_match, binned_sizes, float_close, row_capacity,
                         snapshot_with_sizes)

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS


def _engine():
    from doorman_amd.engine import Engine
    return Engine(0)


@pytest.fixture(scope="module")
def chain():
    e = _engine()
    yield e
    e.close()


def _tick(eng, snap, **kw):
    eng.load(snap)
    eng.apportion(NOW, **kw)
    gets, exp = eng.leases()
    return gets, exp, eng.resources()


def _deterministic(eng, snap, first, label, **kw):
    again = _tick(eng, snap, **kw)
    for x, y in zip(first[:2], again[:2]):
        assert x.tobytes() == y.tobytes(), f"{label}: not deterministic"


def large_sizes(rng, n=12):
    """Large resources around the chunk edges (multiples of 2048 rows, the 4096-row bin
    limit) plus some much larger ones, mixed with every other bin."""
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


@pytest.mark.parametrize("kinds", [(2,), (3,), (0, 1, 2, 3)])
def test_large_against_oracle(chain, kinds):
    """The chain against the oracle; the observed error is reported beside the
    survey's 1e-9 bar and must meet it with the per-client floor too."""
    rng = np.random.default_rng(5 + len(kinds))
    sizes = np.asarray([4097, 8192, 8193, 20000, 33333, 65537], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=kinds)
    gets, exp, res = _tick(chain, snap)
    assert chain.plan_info()["large_chunks"] == int(np.sum(-(-sizes // 2048)))
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, "chain")
    assert_resources_match(snap, res, ref, "chain")
    e = max_err(snap, gets, ref)
    print(f"\nchain kinds={kinds}: max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9


@pytest.mark.parametrize("seed", range(2))
@pytest.mark.parametrize("variant", ["uniform", "hetero", "edge", "recompute", "no_expiry", "learning"])
def test_large_variants_against_oracle(chain, seed, variant):
    """Large resources around the chunk edges mixed with every other bin: heterogeneous
    subclients (the chain's heterogeneous FairShare), IEEE edge wants, recompute mode,
    no expiries, many learning resources; against the oracle, and bit-for-bit
    deterministic run to run."""
    rng = np.random.default_rng(9000 + seed)
    snap = snapshot_with_sizes(rng, large_sizes(rng), hetero=variant == "hetero", edge=variant == "edge",
                               expired_frac=0.0 if variant == "no_expiry" else 0.05,
                               learning_frac=0.5 if variant == "learning" else 0.1)
    rec = variant == "recompute"
    if rec:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            snap.pop(k)
    a = _tick(chain, snap, recompute=rec)
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, a[0], a[1], ref, f"seed={seed} {variant}")
    assert_resources_match(snap, a[2], ref, f"seed={seed} {variant}")
    _deterministic(chain, snap, a, f"seed={seed} {variant}", recompute=rec)


def test_large_resources_at_c2(chain):
    """configs[2]'s large resources (up to 1M rows: 489 chunks of 2048) sampled
    against the oracle with the error reported."""
    snap = W.c2()
    chain.load(snap)
    print(f"\nC2 plan: {chain.plan_info()}")
    chain.apportion(NOW)
    gets, exp = chain.leases()
    so = snap["seg_off"]
    sample = np.asarray([0, 1, 2, 3, 10, 50, 121, 200, 243], dtype=np.int64)  # the largest resources
    sub = W.subset(snap, sample)
    ref = O.apportion(sub, NOW)
    rows = np.concatenate([np.arange(so[r], so[r + 1]) for r in sample])
    assert_leases_match(sub, gets[rows], exp[rows], ref, "C2 large")
    e = max_err(sub, gets[rows], ref)
    print(f"C2 large resources: max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9


def _store_as_snapshot(snap, eng):
    """The device store as it now stands, as an oracle snapshot (running sums included)."""
    st, res = eng.read_store(), eng.resources(safe=False)
    s = dict(snap)
    s.update(has=st["has"], wants=st["wants"], subclients=st["subclients"], expiry_ns=st["expiry_ns"],
             agg_count=res["count"], agg_sum_has=res["sum_has"], agg_sum_wants=res["sum_wants"])
    return s


@pytest.mark.parametrize("cols", ["auto", "alternate"])  # alternate: the speculative chain
def test_large_writeback_ticks_against_oracle(cols):
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
            eng.apportion(now, writeback=True, wb_columns=cols)
            st = eng.read_store()
            live = ref["expiry_ns"] != W.RELEASED
            gets = np.where(live, st["has"], 0.0)
            assert float_close(gets, np.where(live, ref["gets"], 0.0), row_capacity(cur)).all(), f"tick {i} ({step})"
            worst = max(worst, max_err(cur, gets, ref))
        print(f"\nlarge writeback ticks: max |got-ref|/max(|ref|, C_r/n_r) over {len(plan)} ticks = {worst:.3e}")
        assert worst <= 1e-9
    finally:
        eng.close()


@pytest.mark.parametrize("cols", ["auto", "alternate"])  # alternate: the speculative chain
def test_large_writeback_ticks_with_uniform_counts_other_than_one(cols):
    """the steady-state pass A takes each row's count from the last
    writeback tick's live bits and the per-chunk count the map left (Partials::uni),
    not from the subclients column.  Here every large resource holds ONE count other
    than 1 (3 or 7; FairShare and ProportionalShare, whose map also writes the
    subclients column), with writeback ticks back to back (uni used), a non-writeback
    tick between writeback ticks (it must not disturb the state), releases (rows
    marked released, uni kept), and an upsert that gives part of one resource another
    count (the fallback to the column: that resource becomes heterogeneous and goes
    to the heterogeneous chain), each tick against the oracle on the store as it
    stood before it."""
    rng = np.random.default_rng(4343)
    sizes = np.asarray([4097, 6000, 8192, 20000, 65537], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=(3, 2), expired_frac=0.0, learning_frac=0.0,
                               parent_expired_frac=0.0)
    so = snap["seg_off"]
    N = len(snap["wants"])
    counts = np.where(np.arange(len(sizes)) % 2 == 0, 3, 7)
    snap["subclients"] = np.repeat(counts, sizes).astype(np.int64)
    snap["kind"] = np.where(np.arange(len(sizes)) % 2 == 0, W.FAIR_SHARE, W.PROPORTIONAL_SHARE).astype(np.int32)
    snap["expiry_ns"] = np.full(N, NOW + 3600 * W.NS, np.int64)
    snap = W.add_store_sums(snap)
    eng = _engine()
    try:
        eng.load(snap)
        plan = ["same", "same", "same", "peek", "same", "same", "release", "same", "same", "recount", "same", "same"]
        worst = 0.0
        now = NOW
        for i, step in enumerate(plan):
            now += 5 * W.NS
            if step == "release":
                eng.release(rng.choice(N, 300, replace=False).astype(np.int64))
            elif step == "recount":  # half of resource 3's rows take count 2 (its other rows keep 3)
                rows = np.arange(so[3], so[3] + sizes[3] // 2, dtype=np.int64)
                st = eng.read_store()
                eng.upsert(rows, st["has"][rows], st["wants"][rows], np.full(len(rows), 2, np.int64),
                           np.full(len(rows), now + 600 * W.NS, np.int64))
            cur = _store_as_snapshot(snap, eng)
            ref = O.apportion(cur, now)
            if step == "peek":  # a non-writeback tick between writeback ticks
                eng.apportion(now, writeback=False)
                gets, exp = eng.leases()
                assert_leases_match(cur, gets, exp, ref, f"tick {i} (peek)")
                continue
            eng.apportion(now, writeback=True, wb_columns=cols)
            st = eng.read_store()
            live = ref["expiry_ns"] != W.RELEASED
            gets = np.where(live, st["has"], 0.0)
            assert float_close(gets, np.where(live, ref["gets"], 0.0), row_capacity(cur)).all(), f"tick {i} ({step})"
            np.testing.assert_array_equal(st["subclients"][live], np.asarray(cur["subclients"])[live],
                                          err_msg=f"tick {i} ({step}): subclients")
            res = eng.resources(safe=False)
            np.testing.assert_array_equal(res["count"], ref["res_count"], err_msg=f"tick {i} ({step}): count")
            worst = max(worst, max_err(cur, gets, ref))
        print(f"\nuniform counts 3/7: max |got-ref|/max(|ref|, C_r/n_r) over {len(plan)} ticks = {worst:.3e}")
        assert worst <= 1e-9
    finally:
        eng.close()


@pytest.mark.parametrize("redo", ["1", "2"])
def test_speculative_chain_against_the_chain_and_the_oracle(monkeypatch, redo):
    """The speculative chain (k_large_spec: one pass under the totals the resource's
    last tick verified, checked bit for bit per resource; k_large_redo for the
    resources whose totals moved) against the four-launch chain (DM_SPEC_CHAIN=0) and
    the oracle, tick after tick, on large resources of every kind (learning ones
    included) with changes between ticks that move some resources' totals and not
    others': releases, a wants refresh of part of two resources, a capacity change,
    followers lapsing, a non-writeback tick.  Leases match the oracle;
    the two engines' stores hold the same released rows and subclients and running
    sums within the oracle tolerance (their reductions run in different orders); in
    the steady ticks the speculative engine launches no pass of the chain.  redo:
    DM_REDO_LIGHT (1: the redo's light build after a redo-free tick, so the lapse
    tick's redo runs on it; 2: the light build on every tick)."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(8080)
    sizes = np.asarray([4097, 5000, 6000, 8192, 9000, 20000, 65537, 150000, 300, 17, 5], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=(0, 1, 2, 3), expired_frac=0.01, learning_frac=0.0,
                               parent_expired_frac=0.0)
    snap["kind"][:8] = [3, 3, 2, 3, 2, 3, 1, 3]
    snap["learning_end_ns"][:8] = W.INT64_MIN
    snap["learning_end_ns"][2] = NOW + 3600 * W.NS  # one large resource in learning mode
    snap["lease_length_s"][:8] = [40, 600, 600, 600, 35, 600, 600, 600]  # two lapse at the "lapse" tick
    so = np.asarray(snap["seg_off"])
    N = len(snap["wants"])
    cap = np.maximum(snap["capacity"], 1.0)
    monkeypatch.setenv("DM_SPEC_CHAIN", "0")
    chain = Engine(0)
    monkeypatch.delenv("DM_SPEC_CHAIN")
    monkeypatch.setenv("DM_REDO_LIGHT", redo)
    spec = Engine(0)
    try:
        chain.load(snap)
        spec.load(snap)
        spec.set_profiling(True)
        plan = ["same", "same", "same", "same", "release", "same", "same", "wants", "same", "same", "capacity",
                "same", "same", "lapse", "same", "same", "peek", "same", "same"]
        now = NOW
        steady = []
        capacity = snap["capacity"].copy()
        for i, step in enumerate(plan):
            now += (50 if step == "lapse" else 1) * W.NS
            if step == "release":
                rows = rng.choice(N, 300, replace=False).astype(np.int64)
                for e in (chain, spec):
                    e.release(rows)
            elif step == "wants":  # part of resources 1 and 4 (FairShare, ProportionalShare)
                rows = np.concatenate([np.arange(so[1], so[1] + 700), np.arange(so[4], so[4] + 2000)]).astype(np.int64)
                w = rng.uniform(0.0, 3.0, len(rows)) * np.repeat(snap["capacity"], np.diff(so))[rows] / 1000.0
                for e in (chain, spec):
                    e.update_wants(rows, w)
            elif step == "capacity":  # resource 5's capacity halves
                capacity[5] *= 0.5
                c2 = dict(snap)
                c2["capacity"] = capacity
                for e in (chain, spec):
                    e.load_config(c2)
            cur = _store_as_snapshot(snap, spec)
            cur["capacity"] = capacity
            ref = O.apportion(cur, now)
            spec.reset_kernel_times()
            wb = step != "peek"
            # alternate output columns (as on a store beyond the Infinity Cache, C2): the
            # speculative gets must not overwrite has before they are verified
            chain.apportion(now, writeback=wb, wb_columns="alternate")
            spec.apportion(now, writeback=wb, wb_columns="alternate")
            kt = spec.kernel_times()
            steady.append((kt.get("large_spec", (0, 0))[0], kt.get("large_a", (0, 0))[0]))
            if wb:
                st = spec.read_store()
                live = ref["expiry_ns"] != W.RELEASED
                gets = np.where(live, st["has"], 0.0)
                assert float_close(gets, np.where(live, ref["gets"], 0.0), row_capacity(cur)).all(), f"tick {i} ({step})"
                a = chain.read_store()
                np.testing.assert_array_equal(a["expiry_ns"], st["expiry_ns"], err_msg=f"tick {i} ({step})")
                np.testing.assert_array_equal(a["subclients"], st["subclients"], err_msg=f"tick {i} ({step})")
                ra, rb = chain.resources(safe=False), spec.resources(safe=False)
                np.testing.assert_array_equal(ra["count"], rb["count"], err_msg=f"tick {i} ({step})")
                for k in ("sum_has", "sum_wants"):
                    assert float_close(ra[k], rb[k], cap, 1e-12).all(), f"tick {i} ({step}): {k}"
            else:
                gets, exp = spec.leases()
                assert_leases_match(cur, gets, exp, ref, f"tick {i} (peek)")
        # the first tick runs the chain (loaded rows carry explicit expiries); every later
        # writeback tick the speculative launch, never pass A
        assert steady[0] == (0, 1), steady
        assert all(s == (1, 0) for j, s in enumerate(steady[1:], 1) if plan[j] != "peek"), steady
    finally:
        chain.close()
        spec.close()


def test_resource_beyond_the_co_resident_redo_workgroups():
    """A resource with more chunks than 3/4 of the redo workgroups the GPU holds at once
    (plan_info redo_resident_cap: the bound round 4's per-chunk redo had, every chunk of a
    marked resource waiting for the others): the redo by teams (at most kTeamMax
    workgroups per resource) has no such bound, so the store speculates, a wants refresh
    makes the big resource's redo run, and every tick matches the oracle."""
    rng = np.random.default_rng(909)
    probe = _engine()
    try:
        small = snapshot_with_sizes(rng, np.asarray([5000, 20], dtype=np.int64), kinds=(3,), expired_frac=0.0,
                                    learning_frac=0.0, parent_expired_frac=0.0)
        probe.load(small)
        info = probe.plan_info()
        assert info["spec_fits"] == 1
        cap = info["redo_resident_cap"]
    finally:
        probe.close()
    assert 64 <= cap <= 4096, cap
    sizes = np.asarray([cap * 2048 + 1, 6000, 300, 17], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=(3, 2), expired_frac=0.0, learning_frac=0.0, parent_expired_frac=0.0)
    snap["kind"][:2] = [W.FAIR_SHARE, W.PROPORTIONAL_SHARE]
    snap["expiry_ns"] = np.full(len(snap["wants"]), NOW + 3600 * W.NS, np.int64)
    eng = _engine()
    try:
        eng.load(snap)
        assert eng.plan_info()["spec_fits"] == 1
        eng.set_profiling(True)
        now = NOW
        so = np.asarray(snap["seg_off"])
        for i in range(6):
            now += 5 * W.NS
            if i == 4:  # part of the big resource's wants: its speculation fails, the redo runs
                rows = np.arange(so[0], so[0] + 5000, dtype=np.int64)
                eng.update_wants(rows, rng.uniform(0.0, 2.0, len(rows)))
            cur = _store_as_snapshot(snap, eng)
            ref = O.apportion(cur, now)
            eng.reset_kernel_times()
            eng.apportion(now, writeback=True, wb_columns="alternate")
            kt = eng.kernel_times()
            if i >= 1:
                assert kt.get("large_spec", (0, 0))[0] == 1, kt
            st = eng.read_store()
            live = ref["expiry_ns"] != W.RELEASED
            gets = np.where(live, st["has"], 0.0)
            assert float_close(gets, np.where(live, ref["gets"], 0.0), row_capacity(cur)).all(), f"tick {i}"
    finally:
        eng.close()


@pytest.mark.parametrize("redo", ["1", "2"])
def test_back_to_back_async_ticks_against_the_oracle(monkeypatch, redo):
    """What bench.py runs: writeback ticks issued back to back with DM_ASYNC |
    DM_DEFER_JOIN (the class streams join lazily; k_large_redo's build is chosen from a
    host-mapped word the GPU writes ticks behind the host), nothing read in between.
    Segments of such ticks include one where followers lapse (the speculation fails
    without any host call, so the redo runs on the build the heuristic picked), and a
    wants refresh between segments.  After each segment the store equals the oracle's
    ticks applied in order on a host copy."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(6060)
    sizes = np.asarray([4097, 6000, 8192, 20000, 65537, 9000, 300, 17, 5], dtype=np.int64)
    snap = snapshot_with_sizes(rng, sizes, kinds=(2, 3), expired_frac=0.0, learning_frac=0.0,
                               parent_expired_frac=0.0)
    snap["kind"][:6] = [3, 2, 3, 3, 2, 3]
    snap["lease_length_s"][:6] = [600, 30, 600, 25, 600, 600]  # resources 1 and 3 lapse in the long gap
    snap["expiry_ns"] = np.full(len(snap["wants"]), NOW + 3600 * W.NS, np.int64)
    W.add_store_sums(snap)
    so = np.asarray(snap["seg_off"])
    monkeypatch.setenv("DM_REDO_LIGHT", redo)
    eng = Engine(0)
    try:
        eng.load(snap)
        eng.set_profiling(True)
        host = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in snap.items()}
        now = NOW
        segments = [[1, 1, 1], [1, 1, 1, 1], [40, 1, 1], [1, 1]]
        for si, seg in enumerate(segments):
            if si == 3:  # a wants refresh of part of resources 0 and 4 (a synchronous call between segments)
                rows = np.concatenate([np.arange(so[0], so[0] + 900), np.arange(so[4], so[4] + 3000)]).astype(np.int64)
                w = rng.uniform(0.0, 3.0, len(rows)) * np.repeat(snap["capacity"], np.diff(so))[rows] / 1000.0
                eng.update_wants(rows, w)
                live = host["expiry_ns"][rows] != W.RELEASED
                host["wants"][rows] = np.where(live, w, host["wants"][rows])
                W.add_store_sums(host)
            for dt in seg:
                now += dt * W.NS
                eng.apportion(now, writeback=True, asynchronous=True, defer_join=True, wb_columns="alternate")
                ref = O.apportion(host, now)
                live = ref["expiry_ns"] != W.RELEASED
                host["has"] = np.where(live, ref["gets"], 0.0)
                host["wants"] = np.where(live, host["wants"], 0.0)
                host["subclients"] = np.where(live, host["subclients"], 0)
                host["expiry_ns"] = ref["expiry_ns"].copy()
                W.add_store_sums(host)
            eng.sync()
            st = eng.read_store()
            np.testing.assert_array_equal(st["expiry_ns"], host["expiry_ns"], err_msg=f"segment {si}")
            np.testing.assert_array_equal(st["subclients"], host["subclients"], err_msg=f"segment {si}")
            assert float_close(st["has"], host["has"], row_capacity(host)).all(), f"segment {si}"
            res = eng.resources(safe=False)
            np.testing.assert_array_equal(res["count"], host["agg_count"], err_msg=f"segment {si}")
        kt = eng.kernel_times()
        assert kt.get("large_spec", (0, 0))[0] >= 8 and kt.get("large_redo", (0, 0))[0] >= 8, kt
    finally:
        eng.close()
