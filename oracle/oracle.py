"""ctypes binding of the CPU oracle (oracle/doorman_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (doorman_amd/).

The oracle restates go/server/doorman/{store,algorithm,resource}.go; see
doorman_oracle.h for the parity status and the reference lines each function
follows.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

NO_ALGORITHM, STATIC, PROPORTIONAL_SHARE, FAIR_SHARE, LEARN = 0, 1, 2, 3, 4
RELEASED = np.iinfo(np.int64).min
INT64_MAX = np.iinfo(np.int64).max
INT64_MIN = np.iinfo(np.int64).min
NS = 1_000_000_000

# or_resource_cfg (doorman_oracle.h) — natural C alignment
CFG_DTYPE = np.dtype(
    [
        ("kind", np.int32),
        ("capacity", np.float64),
        ("lease_length_s", np.int64),
        ("refresh_interval_s", np.int64),
        ("learning_end_ns", np.int64),
        ("parent_expiry_ns", np.int64),
        ("safe_capacity", np.float64),
    ],
    align=True,
)


class _Lease(ctypes.Structure):
    _fields_ = [
        ("expiry_ns", ctypes.c_int64),
        ("refresh_ns", ctypes.c_int64),
        ("has", ctypes.c_double),
        ("wants", ctypes.c_double),
        ("subclients", ctypes.c_int64),
    ]


class _Request(ctypes.Structure):
    _fields_ = [
        ("client", ctypes.c_int64),
        ("has", ctypes.c_double),
        ("wants", ctypes.c_double),
        ("subclients", ctypes.c_int64),
    ]


class _Snapshot(ctypes.Structure):
    _fields_ = [
        ("n_resources", ctypes.c_int64),
        ("n_leases", ctypes.c_int64),
        ("seg_off", ctypes.c_void_p),
        ("wants", ctypes.c_void_p),
        ("has", ctypes.c_void_p),
        ("subclients", ctypes.c_void_p),
        ("expiry_ns", ctypes.c_void_p),
        ("cfg", ctypes.c_void_p),
        ("agg_count", ctypes.c_void_p),
        ("agg_sum_has", ctypes.c_void_p),
        ("agg_sum_wants", ctypes.c_void_p),
    ]


class _Outputs(ctypes.Structure):
    _fields_ = [
        ("gets", ctypes.c_void_p),
        ("expiry_ns", ctypes.c_void_p),
        ("res_count", ctypes.c_void_p),
        ("res_sum_has", ctypes.c_void_p),
        ("res_sum_wants", ctypes.c_void_p),
        ("res_safe_capacity", ctypes.c_void_p),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, f64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_int32
        L.or_store_new.restype = vp
        L.or_store_new.argtypes = [i64]
        L.or_store_free.argtypes = [vp]
        L.or_store_clone.restype = vp
        L.or_store_clone.argtypes = [vp]
        L.or_store_count.restype = i64
        L.or_store_count.argtypes = [vp]
        L.or_store_sum_has.restype = f64
        L.or_store_sum_has.argtypes = [vp]
        L.or_store_sum_wants.restype = f64
        L.or_store_sum_wants.argtypes = [vp]
        L.or_store_has_client.restype = ctypes.c_int
        L.or_store_has_client.argtypes = [vp, i64]
        L.or_store_get.argtypes = [vp, i64, ctypes.POINTER(_Lease)]
        L.or_store_release.argtypes = [vp, i64]
        L.or_store_assign.argtypes = [vp, i64, i64, i64, f64, f64, i64, i64, ctypes.POINTER(_Lease)]
        L.or_store_put.argtypes = [vp, i64, ctypes.POINTER(_Lease)]
        L.or_store_set_sums.argtypes = [vp, i64, f64, f64]
        L.or_store_clean.restype = i64
        L.or_store_clean.argtypes = [vp, i64]
        L.or_algorithm.restype = ctypes.c_int
        L.or_algorithm.argtypes = [i32, i64, i64, vp, f64, ctypes.POINTER(_Request), i64, ctypes.POINTER(_Lease)]
        L.or_decide.restype = ctypes.c_int
        L.or_decide.argtypes = [vp, vp, ctypes.POINTER(_Request), i64, ctypes.POINTER(_Lease)]
        L.or_aggregate_bands.restype = ctypes.c_int
        L.or_aggregate_bands.argtypes = [vp, vp, i64, ctypes.POINTER(f64), ctypes.POINTER(i64)]
        L.or_apportion_literal.restype = ctypes.c_int
        L.or_apportion_literal.argtypes = [ctypes.POINTER(_Snapshot), i64, ctypes.POINTER(_Outputs)]
        L.or_apportion_closed.restype = ctypes.c_int
        L.or_apportion_closed.argtypes = [ctypes.POINTER(_Snapshot), i64, ctypes.POINTER(_Outputs)]
        L.or_apportion_closed_mt.restype = ctypes.c_int
        L.or_apportion_closed_mt.argtypes = [ctypes.POINTER(_Snapshot), i64, ctypes.POINTER(_Outputs), i32]
        L.or_apportion_literal_rows.restype = i64
        L.or_apportion_literal_rows.argtypes = [ctypes.POINTER(_Snapshot), i64, i64, i64, i64, vp]
        L.or_apportion_literal_sample.restype = i64
        L.or_apportion_literal_sample.argtypes = [ctypes.POINTER(_Snapshot), vp, i64, i64, i64, vp, i32]
        _lib = L
    return _lib


# --------------------------------------------------------------------------
# Go-shaped store / algorithm wrappers (for replaying the reference's tests)
# --------------------------------------------------------------------------
class Lease:
    def __init__(self, l: _Lease):
        self.expiry_ns = l.expiry_ns
        self.refresh_ns = l.refresh_ns
        self.has = l.has
        self.wants = l.wants
        self.subclients = l.subclients

    def is_zero(self) -> bool:  # store.go:62-64
        return self.expiry_ns == 0


class Store:
    """go/server/doorman/store.go leaseStoreImpl over dense client ids."""

    def __init__(self, max_clients: int = 64, _ptr=None):
        self._p = _ptr if _ptr is not None else lib().or_store_new(max_clients)

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.or_store_free(self._p)
            self._p = None

    def clone(self) -> "Store":
        return Store(_ptr=lib().or_store_clone(self._p))

    def count(self) -> int:
        return lib().or_store_count(self._p)

    def sum_has(self) -> float:
        return lib().or_store_sum_has(self._p)

    def sum_wants(self) -> float:
        return lib().or_store_sum_wants(self._p)

    def has_client(self, c: int) -> bool:
        return bool(lib().or_store_has_client(self._p, c))

    def get(self, c: int) -> Lease:
        l = _Lease()
        lib().or_store_get(self._p, c, ctypes.byref(l))
        return Lease(l)

    def release(self, c: int) -> None:
        lib().or_store_release(self._p, c)

    def assign(self, c, lease_length_s, refresh_s, has, wants, sub, now_ns) -> Lease:
        l = _Lease()
        lib().or_store_assign(self._p, c, lease_length_s * NS, refresh_s * NS, has, wants, sub, now_ns, ctypes.byref(l))
        return Lease(l)

    def clean(self, now_ns: int) -> int:
        return lib().or_store_clean(self._p, now_ns)

    def put(self, c, expiry_ns, has, wants, sub, refresh_ns=0) -> None:
        """A stored lease with an explicit expiry (running sums updated as Assign does)."""
        lib().or_store_put(self._p, c, ctypes.byref(_Lease(expiry_ns, refresh_ns, has, wants, sub)))

    def set_sums(self, count, sum_has, sum_wants) -> None:
        """Override the running sums (a snapshot's parity-mode aggregates)."""
        lib().or_store_set_sums(self._p, count, sum_has, sum_wants)


def algorithm(kind, store: Store, capacity, client, has, wants, sub, now_ns=0, lease_length_s=0, refresh_s=0) -> Lease:
    """algorithm.go:44 Algorithm(store, capacity, request) for GetAlgorithm(kind)."""
    q = _Request(client, has, wants, sub)
    l = _Lease()
    rc = lib().or_algorithm(kind, lease_length_s, refresh_s, store._p, capacity, ctypes.byref(q), now_ns, ctypes.byref(l))
    if rc != 0:
        raise ValueError(f"unknown algorithm kind {kind}")
    return Lease(l)


def make_cfg(n, kind=FAIR_SHARE, capacity=100.0, lease_length_s=300, refresh_interval_s=5,
             learning_end_ns=INT64_MIN, parent_expiry_ns=INT64_MAX, safe_capacity=np.nan) -> np.ndarray:
    cfg = np.zeros(n, dtype=CFG_DTYPE)
    cfg["kind"] = kind
    cfg["capacity"] = capacity
    cfg["lease_length_s"] = lease_length_s
    cfg["refresh_interval_s"] = refresh_interval_s
    cfg["learning_end_ns"] = learning_end_ns
    cfg["parent_expiry_ns"] = parent_expiry_ns
    cfg["safe_capacity"] = safe_capacity
    return cfg


def decide(store: Store, cfg_row: np.ndarray, client, has, wants, sub, now_ns) -> Lease:
    """resource.go:100-113 Resource.Decide."""
    cfg = np.ascontiguousarray(cfg_row.reshape(1)).astype(CFG_DTYPE)
    q = _Request(client, has, wants, sub)
    l = _Lease()
    rc = lib().or_decide(store._p, cfg.ctypes.data, ctypes.byref(q), now_ns, ctypes.byref(l))
    if rc != 0:
        raise ValueError("unknown algorithm kind")
    return Lease(l)


def aggregate_bands(wants, num_clients):
    """server.go:850-868; raises ValueError (codes.InvalidArgument) for num_clients < 1."""
    w = np.ascontiguousarray(wants, dtype=np.float64)
    n = np.ascontiguousarray(num_clients, dtype=np.int64)
    wt, st = ctypes.c_double(), ctypes.c_int64()
    if lib().or_aggregate_bands(w.ctypes.data, n.ctypes.data, len(w), ctypes.byref(wt), ctypes.byref(st)) != 0:
        raise ValueError("subclients should be > 0")
    return wt.value, st.value


# --------------------------------------------------------------------------
# Snapshot batch
# --------------------------------------------------------------------------
def _cfg_struct(snap) -> np.ndarray:
    R = len(snap["seg_off"]) - 1
    cfg = np.zeros(R, dtype=CFG_DTYPE)
    for f in CFG_DTYPE.names:
        cfg[f] = snap[f]
    return cfg


def _mk_snapshot(snap, keep):
    def arr(name, dt):
        a = np.ascontiguousarray(snap[name], dtype=dt)
        keep.append(a)
        return a.ctypes.data

    cfg = _cfg_struct(snap)
    keep.append(cfg)
    s = _Snapshot()
    s.n_resources = len(snap["seg_off"]) - 1
    s.n_leases = len(snap["wants"])
    s.seg_off = arr("seg_off", np.int64)
    s.wants = arr("wants", np.float64)
    s.has = arr("has", np.float64)
    s.subclients = arr("subclients", np.int64)
    s.expiry_ns = arr("expiry_ns", np.int64)
    s.cfg = cfg.ctypes.data
    if snap.get("agg_count") is not None:
        s.agg_count = arr("agg_count", np.int64)
        s.agg_sum_has = arr("agg_sum_has", np.float64)
        s.agg_sum_wants = arr("agg_sum_wants", np.float64)
    return s


def apportion(snap: dict, now_ns: int, mode: str = "closed", threads: int = 1) -> dict:
    """Evaluate every row of a snapshot (dict of numpy columns, see
    doorman_amd.workloads) against the frozen store.  mode: 'closed' | 'literal';
    threads > 1 runs the closed form over resources on that many OpenMP threads."""
    keep = []
    s = _mk_snapshot(snap, keep)
    R, N = s.n_resources, s.n_leases
    out = {
        "gets": np.zeros(N, np.float64),
        "expiry_ns": np.zeros(N, np.int64),
        "res_count": np.zeros(R, np.int64),
        "res_sum_has": np.zeros(R, np.float64),
        "res_sum_wants": np.zeros(R, np.float64),
        "res_safe_capacity": np.zeros(R, np.float64),
    }
    o = _Outputs(*[out[k].ctypes.data for k in
                   ("gets", "expiry_ns", "res_count", "res_sum_has", "res_sum_wants", "res_safe_capacity")])
    if mode == "closed" and threads > 1:
        rc = lib().or_apportion_closed_mt(ctypes.byref(s), now_ns, ctypes.byref(o), threads)
    else:
        fn = lib().or_apportion_closed if mode == "closed" else lib().or_apportion_literal
        rc = fn(ctypes.byref(s), now_ns, ctypes.byref(o))
    if rc != 0:
        raise ValueError("unknown algorithm kind in snapshot")
    return out


def apportion_literal_rows(snap: dict, resource: int, row_lo: int, row_hi: int, now_ns: int, gets: np.ndarray) -> int:
    """Literal per-request Decide for rows [row_lo,row_hi) of one resource (CPU baseline sample)."""
    keep = []
    s = _mk_snapshot(snap, keep)
    return lib().or_apportion_literal_rows(ctypes.byref(s), resource, row_lo, row_hi, now_ns, gets.ctypes.data)


def apportion_literal_sample(snap: dict, resources, row_cap: int, now_ns: int, gets: np.ndarray,
                             threads: int = 1) -> int:
    """Literal per-request Decide for the first row_cap rows of each listed resource on
    `threads` OpenMP threads (bench.py cpu_baseline)."""
    keep = []
    s = _mk_snapshot(snap, keep)
    res = np.ascontiguousarray(resources, dtype=np.int64)
    return lib().or_apportion_literal_sample(ctypes.byref(s), res.ctypes.data, len(res), int(row_cap), now_ns,
                                             gets.ctypes.data, int(threads))
