"""Heterogeneous-subclient FairShare (k_general: one threshold per distinct
subclient count, algorithm.go:188-204) against the oracle: the sorted-threshold
bucket pass (up to 256 distinct thresholds, extraExtra = k(T)*T - sum(w < T)) and
the per-threshold passes it falls back to beyond that."""
import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import assert_leases_match, assert_resources_match, row_capacity

pytestmark = pytest.mark.gpu
NOW = W.NOW_NS


@pytest.fixture(scope="module")
def eng():
    from doorman_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def hetero_snapshot(rng, sizes, max_sub, contention=0.8, expired_frac=0.02, dup_frac=0.0):
    """FairShare resources whose clients carry 1..max_sub subclients; most clients want
    more than their share, so most rows reach round 2 (one threshold per distinct
    subclient count)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    R, N = len(sizes), int(sizes.sum())
    sub = rng.integers(1, max_sub + 1, N)
    cap = rng.uniform(500.0, 5000.0, R)
    per = np.repeat(cap / np.maximum(np.add.reduceat(sub, np.r_[0, np.cumsum(sizes)[:-1]]), 1), sizes) * sub
    hi = rng.random(N) < contention
    wants = np.where(hi, rng.uniform(1.0, 6.0, N), rng.uniform(0.0, 1.0, N)) * per
    if dup_frac:
        d = rng.random(N) < dup_frac
        wants[d] = np.round(wants[d], 1)
    has = rng.uniform(0.0, 1.0, N) * per
    exp = NOW + rng.integers(1, 300, N, dtype=np.int64) * W.NS
    dead = rng.random(N) < expired_frac
    exp[dead] = NOW - W.NS
    return W.make_snapshot(sizes, wants, has, sub, exp, np.full(R, 3, np.int32), cap)


def max_err(snap, gets, ref):
    so = snap["seg_off"]
    n_of_row = np.maximum(np.repeat(np.diff(so), np.diff(so)), 1)
    floor = np.abs(row_capacity(snap)) / n_of_row
    live = ref["expiry_ns"] != W.RELEASED
    denom = np.maximum(np.abs(ref["gets"][live]), floor[live])
    return float(np.max(np.abs(gets[live] - ref["gets"][live]) / denom))


@pytest.mark.parametrize("n,max_sub", [(100_000, 150), (100_000, 120), (30_000, 400)])
def test_general_large_resource_many_thresholds(eng, n, max_sub):
    """One resource of n rows with >= 100 distinct subclient counts,
    plus a few small hetero resources; 400 distinct counts take the fallback passes."""
    rng = np.random.default_rng(n + max_sub)
    snap = hetero_snapshot(rng, [n, 50, 3000, 9], max_sub, dup_frac=0.05)
    distinct = len(np.unique(snap["subclients"][:n]))
    assert distinct >= 100
    eng.load(snap)
    eng.apportion(NOW)
    gets, exp = eng.leases()
    res = eng.resources()
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, f"n={n}")
    assert_resources_match(snap, res, ref, f"n={n}")
    e = max_err(snap, gets, ref)
    print(f"\nn={n} distinct subclient counts={distinct}: max |got-ref|/max(|ref|, C_r/n_r) = {e:.3e} (bar 1e-9)")
    assert e <= 1e-9
    eng.apportion(NOW)  # deterministic
    g2, e2 = eng.leases()
    assert g2.tobytes() == gets.tobytes() and e2.tobytes() == exp.tobytes()


@pytest.mark.parametrize("seed", range(3))
def test_general_every_bin_writeback(eng, seed):
    """Heterogeneous resources in every size bin, two writeback ticks (the bucket pass
    reads a store whose decided rows were already written back in place)."""
    rng = np.random.default_rng(700 + seed)
    sizes = [1, 5, 9, 16, 17, 40, 64, 65, 200, 256, 300, 700, 1500, 3000, 4096, 4097, 9000, 20000]
    snap = hetero_snapshot(rng, sizes, 30 + 40 * seed)
    for i in range(2):
        eng.load(snap)
        eng.apportion(NOW + i * W.NS, writeback=True, wb_columns="inplace" if seed % 2 else "alternate")
        gets, exp = eng.leases()
        ref = O.apportion(snap, NOW + i * W.NS)
        assert_leases_match(snap, gets, exp, ref, f"seed={seed} tick={i}")
        st = eng.read_store()
        snap = dict(snap, has=st["has"], wants=st["wants"], subclients=st["subclients"], expiry_ns=st["expiry_ns"])
        W.add_store_sums(snap)


@pytest.mark.parametrize("n,max_sub,nan", [(1_000_000, 150, False), (250_000, 256, False), (60_000, 40, True)])
def test_general_on_the_chain_multi_workgroup(eng, n, max_sub, nan):
    """a large heterogeneous-subclient FairShare resource (a leaf whose
    clients are downstream servers, server.go:850-879) decided by the chunked chain
    (k_large_t / k_large_c_het / k_large_e / k_large_map_het: per-chunk bucket partials
    combined in chunk order) instead of one workgroup.  Against the oracle with the
    observed error printed (bar 1e-12 on this path) and the tick's kernel time; NaN
    wants (no threshold) in one variant; deterministic."""
    rng = np.random.default_rng(n + max_sub)
    snap = hetero_snapshot(rng, [n, 700, 5000], max_sub, dup_frac=0.05)
    if nan:
        snap["wants"][rng.choice(n, 50, replace=False)] = np.nan
        W.add_store_sums(snap)
    eng.load(snap)
    eng.apportion(NOW)
    eng.set_profiling(True)
    eng.reset_kernel_times()
    eng.apportion(NOW)
    kt = eng.kernel_times()
    eng.set_profiling(False)
    gets, exp = eng.leases()
    ref = O.apportion(snap, NOW)
    assert_leases_match(snap, gets, exp, ref, f"n={n}")
    assert_resources_match(snap, eng.resources(), ref, f"n={n}")
    e = max_err(snap, gets, ref)
    ms = sum(v[1] for v in kt.values())
    print(f"\nn={n} distinct={len(np.unique(snap['subclients'][:n]))}: observed error {e:.3e}; "
          f"kernels {ms * 1e3:.0f} us: " + ", ".join(f"{k} {v[1] * 1e3:.0f}" for k, v in kt.items()))
    if not nan:  # decided on the chain (k_general takes the 700-row resource; NaN wants go to it too)
        assert "large_map_het" in kt
    assert e <= 1e-12
    eng.apportion(NOW)
    g2, e2 = eng.leases()
    assert g2.tobytes() == gets.tobytes() and e2.tobytes() == exp.tobytes()
