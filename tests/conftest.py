"""Test configuration: paths to the product package and the oracle, markers.

-m "not gpu": oracle vs golden vectors, host logic (loaders, BVH build, camera,
              tiling), C-ABI exports, gloo multi-rank protocol. No GPU needed.
-m gpu      : HIP kernels vs the oracle (parity proper), through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "triangles-sdf-cpu-raytracing_amd", "tests"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and librtamd.so")


@pytest.fixture(scope="session")
def ref():
    import cpuref
    cpuref.build()
    return cpuref


@pytest.fixture(scope="session")
def rt():
    import rtamd
    rtamd.build()
    return rtamd


@pytest.fixture(scope="session")
def gpu(rt):
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return rt
