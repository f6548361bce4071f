"""CPU checks of the C-ABI boundary: the library builds for gfx950, loads, and
exports every entry point include/doorman_hip.h declares (no GPU needed)."""
import ctypes
import subprocess

import numpy as np
import pytest

from doorman_amd import _lib
from doorman_amd.engine import aggregate_bands


def test_header_declares_expected_entry_points():
    syms = _lib.header_symbols()
    for s in ("dm_create", "dm_destroy", "dm_store_load", "dm_config_load", "dm_apportion", "dm_read_leases",
              "dm_store_upsert", "dm_store_release", "dm_publish_totals", "dm_aggregate_bands"):
        assert s in syms


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    missing = [s for s in _lib.header_symbols() if not hasattr(L, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(_lib.header_symbols()) <= exported


def test_every_header_symbol_has_a_binding():
    assert set(_lib.header_symbols()) == set(_lib._SIGS)


def test_code_object_targets_gfx950():
    """Every offload bundle in the library is a gfx950 code object (host code may name
    other targets: rocPRIM's architecture table, pulled in by hipCUB's sorts)."""
    import re
    data = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets


def test_version_string():
    assert b"gfx950" in _lib.lib().dm_version()


def test_aggregate_bands_matches_server_go():
    """server.go:850-868 (host-side, no device involved)."""
    assert aggregate_bands([200.0] * 5, [1, 2, 3, 4, 5]) == (1000.0, 15)
    with pytest.raises(_lib.DmError) as e:
        aggregate_bands([10.0], [0])
    assert e.value.code == _lib.DM_E_ARGUMENT


def test_null_context_is_an_error_not_a_crash():
    L = _lib.lib()
    assert L.dm_apportion(None, 0, 0) == _lib.DM_E_INVAL
    assert L.dm_sync(None) == _lib.DM_E_INVAL


def test_create_without_gpu_fails_loudly():
    n = ctypes.c_int()
    L = _lib.lib()
    if L.dm_device_count(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    ctx = ctypes.c_void_p()
    rc = L.dm_create(0, ctypes.byref(ctx))
    assert rc < 0 and not ctx.value
    assert L.dm_last_error(None)
