"""ctypes binding of libdoorman_hip.so (the C-ABI in include/doorman_hip.h).

No fallback: if the HIP library is missing or no GPU is visible, calls raise.
Import torch BEFORE this module when both are used in one process, so the
library binds to the HIP runtime torch already loaded (same soname).
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdoorman_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "doorman_hip.h")

DM_OK, DM_E_INVAL, DM_E_HIP, DM_E_STATE, DM_E_KIND, DM_E_RANGE, DM_E_ARGUMENT, DM_E_INTERNAL = 0, -1, -2, -3, -4, -5, -6, -7
DM_HIER_INVALID, DM_HIER_COUNT_RANGE = 1, 2
DM_RCCL_ID_BYTES = 128
DM_WRITEBACK, DM_AGG_RECOMPUTE, DM_ASYNC, DM_WB_INPLACE, DM_WB_ALTERNATE, DM_DEFER_JOIN = 1, 2, 4, 8, 16, 32


class DmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"doorman-hip error {code}: {msg}")
        self.code = code


class Snapshot(ctypes.Structure):
    _fields_ = [
        ("n_resources", ctypes.c_int64),
        ("n_leases", ctypes.c_int64),
        ("seg_off", ctypes.c_void_p),
        ("wants", ctypes.c_void_p),
        ("has", ctypes.c_void_p),
        ("subclients", ctypes.c_void_p),
        ("expiry_ns", ctypes.c_void_p),
        ("agg_count", ctypes.c_void_p),
        ("agg_sum_has", ctypes.c_void_p),
        ("agg_sum_wants", ctypes.c_void_p),
    ]


class StoreBatch(ctypes.Structure):
    """dm_store_batch: one round's refresh (row mask + packed wants), departures, arrivals."""
    _fields_ = [
        ("wants_first_row", ctypes.c_int64), ("wants_nwords", ctypes.c_int64), ("wants_mask", ctypes.c_void_p),
        ("wants_n", ctypes.c_int64), ("wants", ctypes.c_void_p),
        ("release_n", ctypes.c_int64), ("release_rows", ctypes.c_void_p),
        ("upsert_n", ctypes.c_int64), ("upsert_rows", ctypes.c_void_p), ("upsert_has", ctypes.c_void_p),
        ("upsert_wants", ctypes.c_void_p), ("upsert_subclients", ctypes.c_void_p),
        ("upsert_expiry_ns", ctypes.c_void_p), ("upsert_subclients32", ctypes.c_void_p),
        ("upsert_now_ns", ctypes.c_int64),
    ]


class ResourceCfg(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_void_p),
        ("capacity", ctypes.c_void_p),
        ("lease_length_s", ctypes.c_void_p),
        ("refresh_interval_s", ctypes.c_void_p),
        ("learning_end_ns", ctypes.c_void_p),
        ("parent_expiry_ns", ctypes.c_void_p),
        ("safe_capacity", ctypes.c_void_p),
    ]


class KernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("launches", ctypes.c_int64), ("total_ms", ctypes.c_double)]


_lib = None
_variants = {}

_SIGS = {
    "dm_version": (ctypes.c_char_p, []),
    "dm_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "dm_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "dm_destroy": (None, [ctypes.c_void_p]),
    "dm_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "dm_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dm_get_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "dm_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "dm_join": (ctypes.c_int, [ctypes.c_void_p]),
    "dm_stream_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dm_store_update_wants_mask": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                                  ctypes.c_int64, ctypes.c_void_p]),
    "dm_store_load": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Snapshot)]),
    "dm_config_load": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ResourceCfg)]),
    "dm_store_upsert": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 5),
    "dm_store_release": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "dm_store_apply": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dm_store_apply_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dm_store_apply_wait": (ctypes.c_int, [ctypes.c_void_p]),
    "dm_hier_root_tick": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                         ctypes.c_void_p, ctypes.c_int]),
    "dm_host_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "dm_host_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dm_store_update_wants": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "dm_read_store": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "dm_apportion": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint32]),
    "dm_read_leases": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "dm_read_leases_proto": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 3),
    "dm_read_resources": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "dm_aggregate_bands": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "dm_publish_totals": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dm_decide": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 6),
    "dm_read_config": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 7),
    "dm_hier_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "dm_hier_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]),
    "dm_hier_pipeline": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "dm_publish_ring": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "dm_hier_attach": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "dm_hier_step": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "dm_rccl_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "dm_hier_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "dm_hier_comm_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "dm_kernel_class_names": (ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int]),
    "dm_set_profiling": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "dm_kernel_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(KernelTime), ctypes.c_int]),
    "dm_reset_kernel_times": (ctypes.c_int, [ctypes.c_void_p]),
    "dm_plan_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "dm_store_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "dm_store_lost": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "dm_read_leases_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    # round-oriented GetCapacity dispatch (dm_server.cpp)
    "dm_server_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.POINTER(ResourceCfg), ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "dm_server_destroy": (None, [ctypes.c_void_p]),
    "dm_server_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "dm_server_get_capacity": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_double,
                                              ctypes.c_double, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "dm_server_release_capacity": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]),
    "dm_server_tick": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "dm_server_lease": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                       ctypes.POINTER(ctypes.c_double)]),
    "dm_server_resource": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double)]),
    "dm_server_ctx": (ctypes.c_void_p, [ctypes.c_void_p]),
}


def header_symbols() -> list[str]:
    """Every function the public header declares."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(dm_\w+)\s*\(", text, flags=re.M)))


def _bind(path, strict=True):
    """strict: every entry point must exist (the in-tree build); an A/B variant built
    from an older tree may lack newer ones."""
    L = ctypes.CDLL(path)  # RTLD_LOCAL: several builds can coexist in one process (A/B runs)
    for name, (res, args) in _SIGS.items():
        if not strict and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib(path: str | None = None):
    """Load the HIP library (raises if it was not built: there is no CPU fallback).
    `path` selects another build of the same ABI (tools/ab.py)."""
    global _lib
    if path is not None and os.path.abspath(path) != LIB_PATH:
        if path not in _variants:
            _variants[path] = _bind(path, strict=False)
        return _variants[path]
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                               "(make -C doorman_amd/csrc); there is no CPU fallback")
        _lib = _bind(LIB_PATH)
    return _lib


def kernel_class_names() -> list[str]:
    """The kernel classes dm_kernel_times reports (no context or GPU needed)."""
    L = lib()
    n = L.dm_kernel_class_names(None, 0)
    arr = (ctypes.c_char_p * n)()
    check(L.dm_kernel_class_names(arr, n), None, L)
    return [x.decode() for x in arr]


def check(rc: int, ctx=None, L=None) -> int:
    if rc < 0:
        msg = (L or lib()).dm_last_error(ctx)
        raise DmError(rc, msg.decode() if msg else "")
    return rc
