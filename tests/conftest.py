import os
import sys

import pytest
import torch  # noqa: F401  (before gsrt: torch's HIP runtime first, as in bench.py; tests use torch device buffers)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "3dgs-raytrace_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: larger CPU oracle runs")


@pytest.fixture(scope="session")
def ctx():
    import gsrt

    c = gsrt.Context(0)
    yield c
    c.close()
