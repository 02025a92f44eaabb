"""pytest setup: `gpu` marker for tests that need an MI355X (run with -m gpu)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (HIP device)")


@pytest.fixture(scope="session")
def gpu_ctx():
    from odp_amd import gpu
    ctx = gpu.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture
def fresh_cls():
    from odp_amd import cls
    cls.reset()
    yield cls
    cls.reset()
