"""Runs the C++ API test (tests/cpp/test_cxx_api.cpp): the reference-shaped
C++ interface (ipm-zoo_amd/include/ipmz/NumericalOptimization.hpp) on the GPU."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cxx_api():
    exe = os.path.join(REPO, "ipm-zoo_amd", "build", "test_cxx_api")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(REPO, "ipm-zoo_amd"), "cxxtest"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cxx api ok" in r.stdout
