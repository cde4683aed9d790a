import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# A hang in a test ends in 30 s, not the library's 10 min production default
# (mccsCommConfig.timeout_ms); worker processes the tests start inherit it.
os.environ.setdefault("MCCS_TIMEOUT_MS", "30000")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the gpurun box)")
    config.addinivalue_line("markers", "slow: long CPU test")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _ring_unless_direct(request, monkeypatch):
    """Every test runs the ring at every size (the library's one-shot default
    would otherwise take small buckets) unless its module sets
    DIRECT_DEFAULTS = True (the direct kernel's own tests)."""
    if not getattr(request.module, "DIRECT_DEFAULTS", False):
        monkeypatch.setenv("MCCS_ONESHOT_BYTES", "-1")
        monkeypatch.setenv("MCCS_DIRECT_BYTES", "-1")
        monkeypatch.setenv("MCCS_LL_BYTES", "-1")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def lib():
    import mccs_amd

    return mccs_amd.load()
