import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # the host application's explicit BLAS opt-in (triad_amd/blas.py), before any GEMM runs
    from triad_amd import blas
    blas.configure()
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "late: whole-step test run after every other test (see below)")


def pytest_collection_modifyitems(config, items):
    """Whole training-step comparisons (several backbones on concurrent streams, two ranks sharing
    the GPU) run after every kernel / head / config parity test: under `-x` a failure there still
    leaves the rest of the suite's results on record. They fail the run all the same."""
    items.sort(key=lambda it: it.get_closest_marker("late") is not None)
