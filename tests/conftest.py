import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: multi-process / long-running test")
    _parallel_cpu_suite(config)


def _parallel_cpu_suite(config):
    """The CPU suite (``-m "not gpu"``) is dominated by multi-process pipeline
    runs that each keep one or two cores busy: spread the test files over
    RNB_TEST_WORKERS (default 4) pytest-xdist workers when the run did not ask
    for a distribution itself. GPU runs stay in one process (one card, a
    bounded process count on the GPU box)."""
    try:
        import xdist  # noqa: F401
    except ImportError:
        return
    workers = int(os.environ.get("RNB_TEST_WORKERS", "4"))
    if (workers <= 1 or hasattr(config, "workerinput")
            or config.getoption("markexpr", "") != "not gpu"
            or config.getvalue("collectonly") or config.getoption("numprocesses", None)
            or config.getoption("dist", "no") != "no"):
        return
    # xdist's own pytest_configure (trylast) registers the distributed session
    config.option.dist = "load"
    config.option.tx = ["popen"] * workers


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
