"""Shared helpers for the parity tests (HIP path vs the CPU oracle)."""
from __future__ import annotations

import numpy as np

from doorman_amd import workloads as W

# SURVEY.md §8(c) / BASELINE.md: gets within 1e-9 * max(|ref|, capacity_r);
# counts, refresh intervals and expiries bit-exact.
REL_TOL = 1e-9


def row_capacity(snap):
    so = snap["seg_off"]
    return np.repeat(np.asarray(snap["capacity"], dtype=np.float64), so[1:] - so[:-1])


def float_close(got, ref, scale, tol=REL_TOL):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    same = (got == ref) | (np.isnan(got) & np.isnan(ref))
    with np.errstate(invalid="ignore"):
        bound = tol * np.maximum(np.abs(ref), np.abs(scale))
        ok = same | (np.abs(got - ref) <= bound)
    return ok


def assert_leases_match(snap, got_gets, got_exp, ref, label=""):
    np.testing.assert_array_equal(got_exp, ref["expiry_ns"], err_msg=f"{label}: expiry must be bit-exact")
    ok = float_close(got_gets, ref["gets"], row_capacity(snap))
    if not ok.all():
        bad = np.flatnonzero(~ok)[:10]
        raise AssertionError(f"{label}: {int((~ok).sum())} gets out of tolerance, e.g. rows {bad.tolist()}: "
                             f"got {got_gets[bad].tolist()} ref {ref['gets'][bad].tolist()}")


def assert_resources_match(snap, res, ref, label=""):
    np.testing.assert_array_equal(res["count"], ref["res_count"], err_msg=f"{label}: count")
    cap = np.abs(np.asarray(snap["capacity"], dtype=np.float64))
    for k_got, k_ref in (("sum_wants", "res_sum_wants"), ("sum_has", "res_sum_has"),
                         ("safe_capacity", "res_safe_capacity")):
        if k_got not in res:
            continue
        scale = np.maximum(cap, 1.0)
        if k_got == "sum_has":  # includes the tick's delta sum: scale by the magnitudes summed
            scale = np.maximum(scale, W.segment_sums(np.abs(np.nan_to_num(snap["has"], posinf=0, neginf=0)),
                                                     snap["seg_off"]))
        ok = float_close(res[k_got], ref[k_ref], scale)
        if not ok.all():
            bad = np.flatnonzero(~ok)[:10]
            raise AssertionError(f"{label}: {k_got} mismatch at resources {bad.tolist()}: "
                                 f"{res[k_got][bad].tolist()} vs {ref[k_ref][bad].tolist()}")


def binned_sizes(rng, per_bin=3, large=True):
    """Resource sizes that exercise every dispatch bin, incl. empty resources."""
    edges = [(0, 0), (1, 8), (9, 16), (17, 32), (33, 64), (65, 256), (257, 512), (513, 1024), (1025, 2048),
             (2049, 4096)]
    if large:
        edges.append((4097, 13000))
    sizes = []
    for lo, hi in edges:
        sizes += list(rng.integers(lo, hi + 1, per_bin))
    sizes += [8, 9, 16, 17, 32, 33, 64, 65, 128, 129, 256, 257, 512, 513, 1024, 1025, 2048, 2049, 4096]
    sizes += [4, 5, 6, 7, 12, 13, 24, 25, 48, 49, 96, 97, 192, 193]  # the sub-wave shapes' edges (dm_device.h kSubShape*)
    if large:  # chunk edges of the large path (kChunkRows = 2048): 1-row tail, exact multiples
        sizes += [4097, 6144, 8192, 10241]
    rng.shuffle(sizes)
    return np.asarray(sizes, dtype=np.int64)


def snapshot_with_sizes(rng, sizes, kinds=(0, 1, 2, 3), hetero=False, expired_frac=0.05, learning_frac=0.1,
                        parent_expired_frac=0.05, edge=False, now_ns=W.NOW_NS):
    """Like workloads.random_snapshot but with the given resource sizes."""
    R, N = len(sizes), int(np.sum(sizes))
    capacity = rng.choice([0.0, 1.0, 100.0, 1000.0, 12345.678], R) * rng.uniform(0.5, 1.5, R)
    n_of_row = np.maximum(np.repeat(sizes, sizes), 1).astype(np.float64)
    cap_of_row = np.repeat(capacity, sizes)
    wants = rng.uniform(0.0, 3.0, N) * cap_of_row / n_of_row
    ties = rng.random(N) < 0.1
    wants[ties] = np.round(wants[ties])
    has = rng.uniform(0.0, 1.2, N) * cap_of_row / n_of_row
    sub = rng.integers(1, 6, N) if hetero else np.ones(N, np.int64)
    exp = now_ns + rng.integers(0, 300, N, dtype=np.int64) * W.NS
    dead = rng.random(N) < expired_frac
    exp[dead] = now_ns - rng.integers(1, 300, int(dead.sum()), dtype=np.int64) * W.NS
    if edge and N:
        k = max(1, N // 200)
        idx = rng.choice(N, k, replace=False)
        wants[idx] = rng.choice([np.nan, np.inf, -np.inf, -5.0, 0.0, -0.0], k)
    kind = rng.choice(np.asarray(kinds, dtype=np.int32), R)
    learning = np.where(rng.random(R) < learning_frac, now_ns + W.NS, W.INT64_MIN).astype(np.int64)
    parent = np.where(rng.random(R) < parent_expired_frac, now_ns - W.NS, W.INT64_MAX).astype(np.int64)
    safe = np.where(rng.random(R) < 0.5, np.nan, rng.uniform(0, 10, R))
    lease = rng.integers(1, 600, R)
    refresh = rng.integers(1, 60, R)
    return W.make_snapshot(sizes, wants, has, sub, exp, kind, capacity, lease, refresh, learning, parent, safe)
