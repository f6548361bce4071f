"""Snapshot layout helpers and the synthetic workloads of SURVEY.md §8(d).

A *snapshot* is a frozen copy of R resources' lease stores in the columnar
layout the device store uses:

  seg_off            int64[R+1]  CSR offsets: resource r owns rows [seg_off[r], seg_off[r+1])
  wants, has         float64[N]  Lease.Wants / Lease.Has             (store.go:20-36)
  subclients         int64[N]    Lease.Subclients
  expiry_ns          int64[N]    Lease.Expiry as unix nanoseconds
  kind               int32[R]    pb.Algorithm.Kind                   (doorman.proto:139-144)
  capacity           float64[R]  ResourceTemplate.capacity
  lease_length_s     int64[R]    Algorithm.lease_length
  refresh_interval_s int64[R]    Algorithm.refresh_interval
  learning_end_ns    int64[R]    Resource.learningModeEndTime         (resource.go:153-163)
  parent_expiry_ns   int64[R]    Resource.expiryTime (INT64_MAX = nil) (resource.go:62-70)
  safe_capacity      float64[R]  ResourceTemplate.safe_capacity (NaN = unset)
  agg_count, agg_sum_has, agg_sum_wants   the store's running sums (store.go:105-111)

Every row is both a stored lease and that client's refresh request
(has, wants, subclients taken from the row).
"""
from __future__ import annotations

import numpy as np

NO_ALGORITHM, STATIC, PROPORTIONAL_SHARE, FAIR_SHARE = 0, 1, 2, 3
INT64_MAX = np.iinfo(np.int64).max
INT64_MIN = np.iinfo(np.int64).min
RELEASED = INT64_MIN
NS = 1_000_000_000
NOW_NS = 1_790_000_000 * NS  # frozen tick time used by the synthetic workloads

CFG_FIELDS = ("kind", "capacity", "lease_length_s", "refresh_interval_s", "learning_end_ns",
              "parent_expiry_ns", "safe_capacity")


def make_snapshot(seg_sizes, wants, has, subclients, expiry_ns, kind, capacity, lease_length_s=300,
                  refresh_interval_s=5, learning_end_ns=INT64_MIN, parent_expiry_ns=INT64_MAX,
                  safe_capacity=np.nan, aggregates=True) -> dict:
    seg_sizes = np.asarray(seg_sizes, dtype=np.int64)
    R = len(seg_sizes)
    seg_off = np.zeros(R + 1, dtype=np.int64)
    np.cumsum(seg_sizes, out=seg_off[1:])
    N = int(seg_off[-1])

    def col(v, dt, n):
        a = np.asarray(v, dtype=dt)
        return np.ascontiguousarray(np.broadcast_to(a, (n,)) if a.ndim == 0 else a)

    snap = {
        "seg_off": seg_off,
        "wants": col(wants, np.float64, N),
        "has": col(has, np.float64, N),
        "subclients": col(subclients, np.int64, N),
        "expiry_ns": col(expiry_ns, np.int64, N),
        "kind": col(kind, np.int32, R),
        "capacity": col(capacity, np.float64, R),
        "lease_length_s": col(lease_length_s, np.int64, R),
        "refresh_interval_s": col(refresh_interval_s, np.int64, R),
        "learning_end_ns": col(learning_end_ns, np.int64, R),
        "parent_expiry_ns": col(parent_expiry_ns, np.int64, R),
        "safe_capacity": col(safe_capacity, np.float64, R),
    }
    for k in ("wants", "has", "subclients", "expiry_ns"):
        assert len(snap[k]) == N, k
    if aggregates:
        add_store_sums(snap)
    return snap


def segment_sums(values: np.ndarray, seg_off: np.ndarray) -> np.ndarray:
    R = len(seg_off) - 1
    out = np.zeros(R, dtype=values.dtype)
    nz = seg_off[1:] > seg_off[:-1]
    if nz.any():
        with np.errstate(invalid="ignore", over="ignore"):
            out[nz] = np.add.reduceat(values, seg_off[:-1][nz])
    return out


def add_store_sums(snap: dict) -> dict:
    """The store's running sums (count, sumHas, sumWants) as store.Assign leaves them.
    Any rounding order is acceptable: in parity mode both the oracle and the device
    consume these numbers verbatim."""
    so = snap["seg_off"]
    snap["agg_count"] = segment_sums(snap["subclients"], so)
    snap["agg_sum_has"] = segment_sums(snap["has"], so)
    snap["agg_sum_wants"] = segment_sums(snap["wants"], so)
    return snap


def subset(snap: dict, resources) -> dict:
    """Snapshot restricted to the given resource ids (sorted)."""
    resources = np.asarray(resources, dtype=np.int64)
    so = snap["seg_off"]
    sizes = so[resources + 1] - so[resources]
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    # every row of the listed resources, in order (vectorised: no per-resource arange)
    rows = np.arange(int(starts[-1]), dtype=np.int64) + np.repeat(so[resources] - starts[:-1], sizes)
    out = {"seg_off": starts}
    for k in ("wants", "has", "subclients", "expiry_ns"):
        out[k] = np.ascontiguousarray(snap[k][rows])
    for k in CFG_FIELDS:
        out[k] = np.ascontiguousarray(snap[k][resources])
    if "agg_count" in snap:
        for k in ("agg_count", "agg_sum_has", "agg_sum_wants"):
            out[k] = np.ascontiguousarray(snap[k][resources])
    return out


def subset_range(snap: dict, r0: int, r1: int) -> dict:
    """Snapshot restricted to the contiguous resources [r0, r1) (a shard): slices, no
    per-resource gather."""
    so = snap["seg_off"]
    a, z = int(so[r0]), int(so[r1])
    out = {"seg_off": np.ascontiguousarray(so[r0:r1 + 1] - so[r0])}
    for k in ("wants", "has", "subclients", "expiry_ns"):
        out[k] = np.ascontiguousarray(snap[k][a:z])
    for k in CFG_FIELDS + ("agg_count", "agg_sum_has", "agg_sum_wants"):
        if k in snap:
            out[k] = np.ascontiguousarray(snap[k][r0:r1])
    return out


# ---------------------------------------------------------------------------
# SURVEY.md §8(d) synthetic workloads
# ---------------------------------------------------------------------------
def c0(seed=0, now_ns=NOW_NS) -> dict:
    """C0: 1 resource, 1,000 clients, ProportionalShare, capacity 1000."""
    rng = np.random.default_rng(seed)
    n, C = 1000, 1000.0
    wants = rng.uniform(0, 3 * C / n, n)
    has = rng.uniform(0, C / n, n)
    exp = now_ns + rng.integers(1, 300, n) * NS
    return make_snapshot([n], wants, has, 1, exp, PROPORTIONAL_SHARE, C, 300, 5)


def uniform(n_resources, clients, kind=FAIR_SHARE, seed=1, now_ns=NOW_NS, capacity=1000.0,
            expired_frac=0.0) -> dict:
    """C1 / C3 shape: n_resources x clients, wants ~ U(0.5,1.5)*C/n, has = a previous grant."""
    rng = np.random.default_rng(seed)
    N = n_resources * clients
    fair = capacity / clients
    wants = rng.uniform(0.5, 1.5, N) * fair
    has = np.minimum(wants, fair)  # what the previous tick granted (sum_has <= capacity)
    exp = now_ns + rng.integers(1, 300, N, dtype=np.int64) * NS
    if expired_frac > 0:
        dead = rng.random(N) < expired_frac
        exp[dead] = now_ns - rng.integers(1, 300, int(dead.sum()), dtype=np.int64) * NS
    if kind == "mixed":
        kinds = np.where(np.arange(n_resources) % 2 == 0, FAIR_SHARE, PROPORTIONAL_SHARE).astype(np.int32)
    else:
        kinds = kind
    return make_snapshot(np.full(n_resources, clients), wants, has, 1, exp, kinds, capacity, 300, 5)


def uniform_range(n_resources, clients, r0, r1, kind=FAIR_SHARE, seed=3, now_ns=NOW_NS, capacity=1000.0,
                  block=1000) -> dict:
    """Resources [r0, r1) of the n_resources x clients uniform workload (the C1 / C3
    shape), generated block by block -- resource block b from its own generator
    (seed, b) -- so that the shards of a node (hierarchy.partition) together hold
    exactly the store one GPU would hold (configs[3]: one 100M-lease snapshot
    sharded by resource id)."""
    fair = capacity / clients
    wants, exp = [], []
    for b in range(r0 // block, (r1 + block - 1) // block):
        lo, hi = b * block, min((b + 1) * block, n_resources)
        rng = np.random.default_rng([seed, b])
        n = (hi - lo) * clients
        w = rng.uniform(0.5, 1.5, n) * fair
        e = now_ns + rng.integers(1, 300, n, dtype=np.int64) * NS
        a, z = (max(lo, r0) - lo) * clients, (min(hi, r1) - lo) * clients
        wants.append(w[a:z])
        exp.append(e[a:z])
    R = r1 - r0
    w = np.concatenate(wants) if wants else np.zeros(0)
    has = np.minimum(w, fair)  # what the previous tick granted (sum_has <= capacity)
    kinds = (np.where(np.arange(r0, r1) % 2 == 0, FAIR_SHARE, PROPORTIONAL_SHARE).astype(np.int32)
             if kind == "mixed" else kind)
    return make_snapshot(np.full(R, clients), w, has, 1, np.concatenate(exp) if exp else np.zeros(0, np.int64),
                         kinds, capacity, 300, 5)


def c1(seed=1, kind=FAIR_SHARE, now_ns=NOW_NS) -> dict:
    """C1: 10,000 resources x 1,000 clients (10M leases), uniform wants."""
    return uniform(10_000, 1_000, kind=kind, seed=seed, now_ns=now_ns)


def zipf_sizes(n_resources=1_000_000, max_clients=1_000_000) -> np.ndarray:
    rank = np.arange(1, n_resources + 1, dtype=np.float64)
    return np.maximum(1, np.floor(max_clients / rank)).astype(np.int64)


def c2(seed=2, now_ns=NOW_NS, n_resources=1_000_000, max_clients=1_000_000, expired_frac=0.01) -> dict:
    """C2: 1M resources, rank-Zipf clients per resource (1..1M; 13,970,034 leases at full
    size), mixed kinds 40% FS / 40% PS / 10% Static / 10% NoAlgorithm, 5% learning,
    wants lognormal(sigma=1)*C/n_r."""
    rng = np.random.default_rng(seed)
    sizes = zipf_sizes(n_resources, max_clients)
    R, N = len(sizes), int(sizes.sum())
    u = rng.random(R)
    kinds = np.select([u < 0.4, u < 0.8, u < 0.9], [FAIR_SHARE, PROPORTIONAL_SHARE, STATIC],
                      NO_ALGORITHM).astype(np.int32)
    capacity = rng.uniform(100.0, 10_000.0, R)
    learning = np.where(rng.random(R) < 0.05, now_ns + 10 * NS, INT64_MIN).astype(np.int64)
    n_of_row = np.repeat(sizes, sizes).astype(np.float64)
    cap_of_row = np.repeat(capacity, sizes)
    wants = rng.lognormal(0.0, 1.0, N) * cap_of_row / n_of_row
    has = np.minimum(wants, cap_of_row / n_of_row)
    exp = now_ns + rng.integers(1, 300, N, dtype=np.int64) * NS
    if expired_frac > 0:
        dead = rng.random(N) < expired_frac
        exp[dead] = now_ns - rng.integers(1, 300, int(dead.sum()), dtype=np.int64) * NS
    return make_snapshot(sizes, wants, has, 1, exp, kinds, capacity, 300, 5, learning_end_ns=learning)


def random_snapshot(rng, n_resources, max_clients, kinds=(0, 1, 2, 3), hetero=False, expired_frac=0.1,
                    learning_frac=0.1, parent_expired_frac=0.05, edge=False, now_ns=NOW_NS) -> dict:
    """Randomised parity snapshot: ragged segments (including empty ones), all
    kinds, expiries, learning mode, parent-lease expiry and optional IEEE edges."""
    sizes = rng.integers(0, max_clients + 1, n_resources)
    R, N = n_resources, int(sizes.sum())
    capacity = rng.choice([0.0, 1.0, 100.0, 1000.0, 12345.678], R) * rng.uniform(0.5, 1.5, R)
    n_of_row = np.maximum(np.repeat(sizes, sizes), 1).astype(np.float64)
    cap_of_row = np.repeat(capacity, sizes)
    wants = rng.uniform(0.0, 3.0, N) * cap_of_row / n_of_row
    # exact small integers and ties against the equal share
    ties = rng.random(N) < 0.15
    wants[ties] = np.round(wants[ties])
    has = rng.uniform(0.0, 1.2, N) * cap_of_row / n_of_row
    sub = rng.integers(1, 6, N) if hetero else np.ones(N, np.int64)
    exp = now_ns + rng.integers(0, 300, N, dtype=np.int64) * NS
    dead = rng.random(N) < expired_frac
    exp[dead] = now_ns - rng.integers(1, 300, int(dead.sum()), dtype=np.int64) * NS
    exact = rng.random(N) < 0.02  # expiry == now: not After(now) -> still live
    exp[exact] = now_ns
    if edge and N > 0:
        k = max(1, N // 50)
        idx = rng.choice(N, k, replace=False)
        wants[idx] = rng.choice([np.nan, np.inf, -np.inf, -5.0, 0.0, -0.0], k)
    kind = rng.choice(np.asarray(kinds, dtype=np.int32), R)
    learning = np.where(rng.random(R) < learning_frac, now_ns + NS, INT64_MIN).astype(np.int64)
    parent = np.where(rng.random(R) < parent_expired_frac, now_ns - NS, INT64_MAX).astype(np.int64)
    safe = np.where(rng.random(R) < 0.5, np.nan, rng.uniform(0, 10, R))
    lease = rng.integers(1, 600, R)
    refresh = rng.integers(1, 60, R)
    return make_snapshot(sizes, wants, has, sub, exp, kind, capacity, lease, refresh, learning, parent, safe)


def rows_to_mask(rows, n_rows: int, first_row: int = 0) -> np.ndarray:
    """Row mask of dm_store_update_wants_mask: bit j of word w is row first_row + 64 w + j."""
    nwords = (n_rows + 63) // 64
    bits = np.zeros(nwords * 64, np.uint8)
    bits[np.asarray(rows, np.int64) - first_row] = 1
    return np.packbits(bits, bitorder="little").view(np.uint64)
