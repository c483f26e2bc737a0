"""Shared pytest setup.

Markers:
  gpu — needs an MI355X (the HIP path through libhipann.so).  The driver runs `-m gpu` on the GPU
        box and `-m "not gpu"` here; CPU tests never call compute entry points of the library.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU (HIP path through libhipann.so)")


@pytest.fixture(scope="session")
def hipann_mod():
    import hipann

    hipann.build()
    return hipann


@pytest.fixture(scope="session")
def gpu(hipann_mod):
    """The loaded HIP library; fails (does not skip) when the GPU path is missing — a GPU test that
    silently skipped would hide a missing native path."""
    assert hipann_mod.is_available(), "libhipann.so loaded but no gfx950 HIP device is available"
    return hipann_mod


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O
