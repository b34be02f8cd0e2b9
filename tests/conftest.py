import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "f110-mpc_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP path")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o

    o.build()
    return o


@pytest.fixture(scope="session")
def capi():
    # torch ships its own HIP runtime next to the system one libf110qp.so links: the runtime that
    # initialises first owns the device, and torch's only comes up if it is first
    try:
        import torch

        torch.cuda.is_available()
    except ImportError:
        pass
    from f110qp import capi as c

    c.load()
    return c


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch.device("cuda", 0)


@pytest.fixture
def knob(capi, monkeypatch):
    """Set a create-time F110QP_* test knob (F110QP_LANE_SEG=4, ...) for the rest of the test and
    route the test's solvers to the test build (lib_test/libf110qp.so), the only library that reads
    them: the product library reads no environment variable (f110qp_api.cpp, test_hooks)."""
    monkeypatch.setattr(capi, "USE_TEST_BUILD", True)

    def set_knob(name, value):
        assert name.startswith("F110QP_"), name
        monkeypatch.setenv(name, str(value))

    return set_knob
