"""Round-oriented GetCapacity / ReleaseCapacity over the device-resident store
(dm_server_* in include/doorman_hip.h, doorman_amd/csrc/dm_server.cpp).

Mirrors the reference server's request path (go/server/doorman/server.go:668-817,
resource.go:100-113): a round's ResourceRequests are queued, then decided by one
dm_server_tick in queue order (dm_decide: each request sees the Assigns of the
requests before it on its resource, as res.mu serialises the reference's calls);
each ticket gets the lease GetCapacity would put in its response (capacity,
expiry_time in unix seconds, refresh_interval, safe_capacity).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .engine import CFG_FIELDS, _c, _ptr


@dataclass
class Lease:
    """pb.Lease of a ResourceResponse plus its SafeCapacity (server.go:783-796)."""
    capacity: float
    expiry_time: int
    refresh_interval: int
    safe_capacity: float


class ServerError(_lib.DmError):
    pass


class TickServer:
    def __init__(self, resources: dict, device: int = 0, slots: int = 8):
        """resources: id -> dict(kind, capacity, lease_length_s, refresh_interval_s,
        learning_end_ns, parent_expiry_ns, safe_capacity) — the resolved templates
        (the reference's LoadConfig + findConfigForResource outcome)."""
        self._L = _lib.lib()
        ids = list(resources)
        R = len(ids)
        defaults = {"lease_length_s": 300, "refresh_interval_s": 5, "learning_end_ns": np.iinfo(np.int64).min,
                    "parent_expiry_ns": np.iinfo(np.int64).max, "safe_capacity": np.nan}
        dtypes = {"kind": np.int32, "capacity": np.float64, "lease_length_s": np.int64,
                  "refresh_interval_s": np.int64, "learning_end_ns": np.int64, "parent_expiry_ns": np.int64,
                  "safe_capacity": np.float64}
        self._keep = {f: _c([resources[i].get(f, defaults.get(f)) for i in ids], dtypes[f]) for f in CFG_FIELDS}
        cfg = _lib.ResourceCfg(*[_ptr(self._keep[f]) for f in CFG_FIELDS])
        self._ids = (ctypes.c_char_p * max(R, 1))(*[i.encode() for i in ids])
        self._srv = ctypes.c_void_p()
        rc = self._L.dm_server_create(device, R, self._ids, ctypes.byref(cfg), slots, ctypes.byref(self._srv))
        if rc < 0:
            raise ServerError(rc, self._L.dm_last_error(None).decode())

    def close(self):
        if self._srv:
            self._L.dm_server_destroy(self._srv)
            self._srv = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc < 0:
            raise ServerError(rc, (self._L.dm_server_last_error(self._srv) or b"").decode())
        return rc

    def get_capacity(self, client: str, resource: str, has: float, wants: float, subclients: int = 1) -> int:
        """Queue one ResourceRequest; returns the ticket of its lease in the next tick."""
        t = ctypes.c_int64()
        self._chk(self._L.dm_server_get_capacity(self._srv, client.encode(), resource.encode(), float(has),
                                                 float(wants), int(subclients), ctypes.byref(t)))
        return t.value

    def release_capacity(self, client: str, resource: str):
        self._chk(self._L.dm_server_release_capacity(self._srv, client.encode(), resource.encode()))

    def tick(self, now_ns: int):
        self._chk(self._L.dm_server_tick(self._srv, int(now_ns)))

    def lease(self, ticket: int) -> Lease:
        c, e, r, s = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        self._chk(self._L.dm_server_lease(self._srv, ticket, ctypes.byref(c), ctypes.byref(e), ctypes.byref(r),
                                          ctypes.byref(s)))
        return Lease(c.value, e.value, r.value, s.value)

    def resource(self, resource: str) -> dict:
        n, cnt, sh, sw = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        self._chk(self._L.dm_server_resource(self._srv, resource.encode(), ctypes.byref(n), ctypes.byref(cnt),
                                             ctypes.byref(sh), ctypes.byref(sw)))
        return {"clients": n.value, "count": cnt.value, "sum_has": sh.value, "sum_wants": sw.value}
