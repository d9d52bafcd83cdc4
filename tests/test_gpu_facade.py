"""The C++ façade (include/eslam_gpu.hpp, the reference's EmbodiedSlamFilter /
PoseEstimator class API over the C ABI) runs on the GPU and equals the raw ABI."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_facade():
    sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
    import build_lib
    exe = build_lib.build_facade_test(verbose=False)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade OK" in r.stdout
