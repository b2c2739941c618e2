import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """GPU sessions: let torch initialise its HIP runtime before the engine's
    library does.  Some tests hand torch tensors (pinned host memory, device
    buffers) to the engine; with the engine's HIP runtime initialised first,
    torch's own initialisation in the same process then found no device (seen
    when a subset of the GPU tests ran without an earlier torch user)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running parity case")


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(TESTS, "golden")

    def load(name):
        with open(os.path.join(d, name)) as f:
            return json.load(f)

    return load


_POINTS = {}


@pytest.fixture(scope="session")
def points():
    """fixed_points(group, n) of the engine's host helper, cached for the session
    (G2 n = 2^20 takes seconds on the host and is used by several modules)."""
    def get(group, n):
        key = (group, n)
        if key not in _POINTS:
            import msm_blst_amd as m
            _POINTS[key] = m.fixed_points(group, n)
        return _POINTS[key]
    return get
