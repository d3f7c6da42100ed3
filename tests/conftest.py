import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "rl-rust_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU-only oracle runs")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    oracle_ffi.build()
    return oracle_ffi


@pytest.fixture(scope="session")
def rl():
    import rlamd
    rlamd.lib()
    return rlamd
