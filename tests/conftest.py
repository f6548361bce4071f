import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# torch first: libdoorman_hip then binds to the HIP runtime torch loads, exactly as
# in bench.py (one HIP runtime per process).
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
