import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    oracle_ffi.build()
    return oracle_ffi


@pytest.fixture(scope="session")
def gpu_mod():
    """the product wrapper over libeslam_gpu.so (fails loudly when the library is missing)"""
    import eslam_amd
    eslam_amd.load_library()
    return eslam_amd
