"""doorman_amd — MI355X-native batched lease apportionment for Doorman.

The engine (device-resident columnar LeaseStore, size-binned gfx950 kernels,
C-ABI) is libdoorman_hip.so, built from doorman_amd/csrc; this package is its
Python binding plus the synthetic workloads of SURVEY.md §8(d).  Nothing here
computes a lease on the CPU: without the HIP library every engine call raises.
"""
from .workloads import (FAIR_SHARE, NO_ALGORITHM, PROPORTIONAL_SHARE, STATIC, NOW_NS, NS, RELEASED,  # noqa: F401
                        make_snapshot)

__all__ = ["Engine", "aggregate_bands", "device_count", "make_snapshot", "NO_ALGORITHM", "STATIC",
           "PROPORTIONAL_SHARE", "FAIR_SHARE", "RELEASED"]


def __getattr__(name):
    if name in ("Engine", "aggregate_bands", "device_count"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
