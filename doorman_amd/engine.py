"""Python handle on one device context of the C-ABI (include/doorman_hip.h).

This is a thin binding used by tests and bench.py; the store, the planner and
the kernels live in libdoorman_hip.so.  Method names follow the reference's
LeaseStore / Algorithm surface (go/server/doorman/store.go:68-103,
algorithm.go:44) where one exists.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib
from .workloads import CFG_FIELDS

_BIN_NAMES = ("small_tiles", "sub16x4", "sub32x4", "wave64x4", "block128x4", "block128x8", "block256x8",
              "block2k4k", "sub8x2", "sub16x2", "large_resources", "large_chunks", "leases", "bin_shapes",
              "redo_resident_cap", "spec_fits", "aux_own_queues", "stream_parts", "queue_perm")


def _ptr(a):
    return None if a is None else a.ctypes.data


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class Engine:
    """One GPU context owning a device-resident columnar lease store."""

    def __init__(self, device: int = 0, lib_path: str | None = None):
        self._L = _lib.lib(lib_path)
        self._ctx = ctypes.c_void_p()
        check(self._L.dm_create(device, ctypes.byref(self._ctx)), None, self._L)
        self.device = device
        self.n_resources = 0
        self.n_leases = 0
        self.seg_off = np.zeros(1, np.int64)
        self._pinned = []

    # -- lifetime --
    def host_empty(self, n: int, dtype=np.float64) -> np.ndarray:
        """A page-locked host array (dm_host_alloc), for update batches that should cross
        PCIe by DMA at full rate.  Valid until close()."""
        dtype = np.dtype(dtype)
        nbytes = max(int(n), 1) * dtype.itemsize
        ptr = ctypes.c_void_p()
        self._chk(self._L.dm_host_alloc(self._ctx, nbytes, ctypes.byref(ptr)))
        self._pinned.append(ptr.value)
        buf = (ctypes.c_byte * nbytes).from_address(ptr.value)
        return np.frombuffer(buf, dtype=dtype, count=int(n))

    def close(self):
        if self._ctx:
            for ptr in getattr(self, "_pinned", []):
                self._L.dm_host_free(self._ctx, ctypes.c_void_p(ptr))
            self._pinned = []
            self._L.dm_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc):
        return check(rc, self._ctx, self._L)

    @property
    def stream(self) -> int:
        return self._L.dm_get_stream(self._ctx) or 0

    def set_stream(self, stream_ptr: int | None):
        self._chk(self._L.dm_set_stream(self._ctx, stream_ptr))

    def sync(self):
        self._chk(self._L.dm_sync(self._ctx))

    def join(self):
        """dm_join: order deferred ticks before later work on the context stream."""
        self._chk(self._L.dm_join(self._ctx))

    def stream_wait(self, hip_stream: int):
        """dm_stream_wait: order hip_stream after the work enqueued so far on this engine."""
        self._chk(self._L.dm_stream_wait(self._ctx, ctypes.c_void_p(hip_stream)))

    # -- LeaseStore --
    def load(self, snap: dict):
        """NewLeaseStore + Assign of every row (store.go:114,153) and the resolved config."""
        self.load_store(snap)
        self.load_config(snap)

    def load_store(self, snap: dict):
        keep = {
            "seg_off": _c(snap["seg_off"], np.int64),
            "wants": _c(snap["wants"], np.float64),
            "has": _c(snap["has"], np.float64),
            "subclients": _c(snap["subclients"], np.int64),
            "expiry_ns": _c(snap["expiry_ns"], np.int64),
        }
        have = snap.get("agg_count") is not None
        if have:
            keep["agg_count"] = _c(snap["agg_count"], np.int64)
            keep["agg_sum_has"] = _c(snap["agg_sum_has"], np.float64)
            keep["agg_sum_wants"] = _c(snap["agg_sum_wants"], np.float64)
        s = _lib.Snapshot()
        s.n_resources = len(keep["seg_off"]) - 1
        s.n_leases = len(keep["wants"])
        for k in ("seg_off", "wants", "has", "subclients", "expiry_ns"):
            setattr(s, k, _ptr(keep[k]))
        if have:
            s.agg_count = _ptr(keep["agg_count"])
            s.agg_sum_has = _ptr(keep["agg_sum_has"])
            s.agg_sum_wants = _ptr(keep["agg_sum_wants"])
        self._chk(self._L.dm_store_load(self._ctx, ctypes.byref(s)))
        self.n_resources, self.n_leases = s.n_resources, s.n_leases
        self.seg_off = keep["seg_off"].copy()  # the table layout (host copy)

    def load_config(self, snap: dict):
        R = len(snap["kind"])
        keep = {
            "kind": _c(snap["kind"], np.int32),
            "capacity": _c(snap["capacity"], np.float64),
            "lease_length_s": _c(snap["lease_length_s"], np.int64),
            "refresh_interval_s": _c(snap["refresh_interval_s"], np.int64),
            "learning_end_ns": _c(snap["learning_end_ns"], np.int64),
            "parent_expiry_ns": _c(snap["parent_expiry_ns"], np.int64),
            "safe_capacity": _c(snap["safe_capacity"], np.float64),
        }
        cfg = _lib.ResourceCfg(*[_ptr(keep[k]) for k in CFG_FIELDS])
        self._chk(self._L.dm_config_load(self._ctx, R, ctypes.byref(cfg)))

    def upsert(self, rows, has, wants, subclients, expiry_ns):
        """Assign on existing rows (store.go:153-167)."""
        rows = _c(rows, np.int64)
        a = [_c(has, np.float64), _c(wants, np.float64), _c(subclients, np.int64), _c(expiry_ns, np.int64)]
        self._chk(self._L.dm_store_upsert(self._ctx, len(rows), _ptr(rows), *[_ptr(x) for x in a]))

    def update_wants(self, rows, wants):
        """Refresh that only changes wants (store.go:153-167, narrow form)."""
        rows, wants = _c(rows, np.int64), _c(wants, np.float64)
        self._chk(self._L.dm_store_update_wants(self._ctx, len(rows), _ptr(rows), _ptr(wants)))

    def update_wants_mask(self, mask, wants, first_row: int = 0):
        """update_wants with the rows as a bit mask (uint64 words; bit j of word w is row
        first_row + 64 w + j) and the values packed in ascending row order."""
        mask, wants = _c(mask, np.uint64), _c(wants, np.float64)
        self._chk(self._L.dm_store_update_wants_mask(self._ctx, int(first_row), len(mask), _ptr(mask), len(wants),
                                                     _ptr(wants)))

    def apply(self, wants_mask=None, wants=None, release_rows=None, upsert=None, wants_first_row: int = 0,
              now_ns: int | None = None, asynchronous: bool = False):
        """dm_store_apply: one round's refresh (row mask + packed wants), departures and
        arrivals (upsert = (rows, has, wants, subclients, expiry_ns)) in one call.
        Narrow arrivals: has None (= 0), subclients as int32 (sent as 4 B), expiry_ns None
        (= now_ns + the resource's lease length: now_ns is then required).
        asynchronous: dm_store_apply_async -- enqueued, not waited for; the arrays are kept
        alive here until the batch is retired (apply_wait, or two batches later), and a
        rejected batch raises from the call that retires it."""
        if upsert is not None and upsert[4] is None and now_ns is None:
            raise ValueError("arrivals without expiries need now_ns (their expiry is now_ns + lease length)")
        keep = []

        def col(a, dt):
            a = _c(a, dt)
            keep.append(a)
            return a

        b = _lib.StoreBatch()
        if wants_mask is not None:
            m, w = col(wants_mask, np.uint64), col(wants if wants is not None else [], np.float64)
            b.wants_first_row, b.wants_nwords, b.wants_mask = int(wants_first_row), len(m), _ptr(m)
            b.wants_n, b.wants = len(w), _ptr(w)
        if release_rows is not None:
            r = col(release_rows, np.int64)
            b.release_n, b.release_rows = len(r), _ptr(r)
        if upsert is not None:
            rows, has, wv, sub, exp = upsert
            rows = col(rows, np.int64)
            b.upsert_n, b.upsert_rows = len(rows), _ptr(rows)
            b.upsert_has = None if has is None else _ptr(col(has, np.float64))
            b.upsert_wants = _ptr(col(wv, np.float64))
            if np.asarray(sub).dtype == np.int32:
                b.upsert_subclients32 = _ptr(col(sub, np.int32))
            else:
                b.upsert_subclients = _ptr(col(sub, np.int64))
            b.upsert_expiry_ns = None if exp is None else _ptr(col(exp, np.int64))
            b.upsert_now_ns = int(now_ns or 0)
        if not asynchronous:
            self._chk(self._L.dm_store_apply(self._ctx, ctypes.byref(b)))
            return
        self._chk(self._L.dm_store_apply_async(self._ctx, ctypes.byref(b)))
        # the library reads these columns until it retires the batch (at most two
        # batches in flight): keep the last three batches' arrays alive
        self._async_keep = (getattr(self, "_async_keep", []) + [keep])[-3:]

    def apply_wait(self):
        """dm_store_apply_wait: retire every in-flight asynchronous batch (raises for the
        first rejected one)."""
        try:
            self._chk(self._L.dm_store_apply_wait(self._ctx))
        finally:
            self._async_keep = []

    def release(self, rows):
        """Release (store.go:142-151)."""
        rows = _c(rows, np.int64)
        self._chk(self._L.dm_store_release(self._ctx, len(rows), _ptr(rows)))

    def read_store(self, off: int = 0, n: int | None = None) -> dict:
        n = self.n_leases - off if n is None else n
        out = {"has": np.empty(n), "wants": np.empty(n), "subclients": np.empty(n, np.int64),
               "expiry_ns": np.empty(n, np.int64)}
        self._chk(self._L.dm_read_store(self._ctx, off, n, _ptr(out["has"]), _ptr(out["wants"]),
                                      _ptr(out["subclients"]), _ptr(out["expiry_ns"])))
        return out

    # -- the batch algorithm --
    def apportion(self, now_ns: int, writeback: bool = False, recompute: bool = False, asynchronous: bool = False,
                  wb_columns: str = "auto", defer_join: bool = False):
        """wb_columns: "auto", "inplace" or "alternate" (DM_WB_INPLACE / DM_WB_ALTERNATE);
        defer_join (with asynchronous): DM_DEFER_JOIN."""
        flags = ((_lib.DM_WRITEBACK if writeback else 0) | (_lib.DM_AGG_RECOMPUTE if recompute else 0)
                 | (_lib.DM_ASYNC if asynchronous else 0) | (_lib.DM_DEFER_JOIN if defer_join else 0)
                 | {"auto": 0, "inplace": _lib.DM_WB_INPLACE, "alternate": _lib.DM_WB_ALTERNATE}[wb_columns])
        self._chk(self._L.dm_apportion(self._ctx, int(now_ns), flags))

    def decide(self, now_ns: int, rows, has, wants, subclients):
        """dm_decide: Resource.Decide for each request of a round, in order, each seeing
        the Assigns of the requests before it on its resource (rows[k] = the client's
        row, or a free row of its resource for a new client; a row may repeat);
        returns (gets, expiry_ns).  The device store is not changed."""
        rows = _c(rows, np.int64)
        a = [_c(has, np.float64), _c(wants, np.float64), _c(subclients, np.int64)]
        gets, exp = np.empty(len(rows)), np.empty(len(rows), np.int64)
        self._chk(self._L.dm_decide(self._ctx, int(now_ns), len(rows), _ptr(rows), *[_ptr(x) for x in a], _ptr(gets),
                                    _ptr(exp)))
        return gets, exp

    def leases(self, off: int = 0, n: int | None = None):
        n = self.n_leases - off if n is None else n
        gets, exp = np.empty(n), np.empty(n, np.int64)
        self._chk(self._L.dm_read_leases(self._ctx, off, n, _ptr(gets), _ptr(exp)))
        return gets, exp

    def leases_rows(self, rows):
        """dm_read_leases_rows: the last tick's leases of scattered rows (gathered on the device)."""
        rows = _c(rows, np.int64)
        gets, exp = np.empty(len(rows)), np.empty(len(rows), np.int64)
        self._chk(self._L.dm_read_leases_rows(self._ctx, len(rows), _ptr(rows), _ptr(gets), _ptr(exp)))
        return gets, exp

    def leases_proto(self, off: int = 0, n: int | None = None):
        n = self.n_leases - off if n is None else n
        cap, exp, ref = np.empty(n), np.empty(n, np.int64), np.empty(n, np.int64)
        self._chk(self._L.dm_read_leases_proto(self._ctx, off, n, _ptr(cap), _ptr(exp), _ptr(ref)))
        return cap, exp, ref

    def resources(self, r0: int = 0, n: int | None = None, safe: bool = True) -> dict:
        n = self.n_resources - r0 if n is None else n
        out = {"count": np.empty(n, np.int64), "sum_has": np.empty(n), "sum_wants": np.empty(n)}
        if safe:
            out["safe_capacity"] = np.empty(n)
        self._chk(self._L.dm_read_resources(self._ctx, r0, n, _ptr(out["count"]), _ptr(out["sum_has"]),
                                          _ptr(out["sum_wants"]), _ptr(out.get("safe_capacity"))))
        return out

    def config(self, r0: int = 0, n: int | None = None) -> dict:
        """dm_read_config: the per-resource configuration the device holds (CFG_FIELDS columns)."""
        n = self.n_resources - r0 if n is None else n
        out = {"kind": np.empty(n, np.int32), "capacity": np.empty(n), "lease_length_s": np.empty(n, np.int64),
               "refresh_interval_s": np.empty(n, np.int64), "learning_end_ns": np.empty(n, np.int64),
               "parent_expiry_ns": np.empty(n, np.int64), "safe_capacity": np.empty(n)}
        self._chk(self._L.dm_read_config(self._ctx, r0, n, *[_ptr(out[k]) for k in CFG_FIELDS]))
        return out

    def publish_totals(self, dev_ptr: int):
        """{SumWants, Count} per resource into a 16 B x R device buffer (server.go:234-255)."""
        self._chk(self._L.dm_publish_totals(self._ctx, ctypes.c_void_p(dev_ptr)))

    # -- profiling --
    def set_profiling(self, on: bool):
        self._chk(self._L.dm_set_profiling(self._ctx, 1 if on else 0))

    def kernel_times(self) -> dict:
        cap = 64
        arr = (_lib.KernelTime * cap)()
        n = self._chk(self._L.dm_kernel_times(self._ctx, arr, cap))
        if n > cap:
            raise RuntimeError(f"dm_kernel_times reports {n} kernel classes, more than {cap}")
        return {arr[i].name.decode(): (arr[i].launches, arr[i].total_ms) for i in range(n) if arr[i].launches}

    def reset_kernel_times(self):
        self._chk(self._L.dm_reset_kernel_times(self._ctx))

    def plan_info(self) -> dict:
        arr = (ctypes.c_int64 * 32)()
        n = self._chk(self._L.dm_plan_info(self._ctx, arr, 32))
        return {_BIN_NAMES[i]: int(arr[i]) for i in range(min(n, len(_BIN_NAMES)))}

    def store_lost(self) -> bool:
        """dm_store_lost: a device-side invariant failed; ticks and updates refuse the store
        until it is reloaded, the read calls still work on it."""
        v = ctypes.c_int(0)
        self._chk(self._L.dm_store_lost(self._ctx, ctypes.byref(v)))
        return bool(v.value)

    def store_stats(self) -> dict:
        """dm_store_stats: dense resources (read at 24 B per lease) and their rows,
        resources that may hold explicit expiries, resources."""
        arr = (ctypes.c_int64 * 4)()
        self._chk(self._L.dm_store_stats(self._ctx, arr, 4))
        return {"dense_resources": int(arr[0]), "dense_leases": int(arr[1]), "explicit_resources": int(arr[2]),
                "resources": int(arr[3])}


def device_count() -> int:
    n = ctypes.c_int()
    rc = lib().dm_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def aggregate_bands(wants, num_clients):
    """GetServerCapacity band sums (server.go:850-868); DmError(DM_E_ARGUMENT) if num_clients < 1."""
    w, nc = _c(wants, np.float64), _c(num_clients, np.int64)
    wt, st = ctypes.c_double(), ctypes.c_int64()
    check(lib().dm_aggregate_bands(_ptr(w), _ptr(nc), len(w), ctypes.byref(wt), ctypes.byref(st)))
    return wt.value, st.value
