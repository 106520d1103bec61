import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "allreduce-over-mpi_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "capture_runtime_limit: a graph-capture shape the HIP runtime crashes on "
                                       "(SIGSEGV in hipStreamEndCapture, DESIGN §4); runs only with "
                                       "FTAR_RUN_CAPTURE_LIMITS=1")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("FTAR_RUN_CAPTURE_LIMITS") == "1":
        return
    skip = pytest.mark.skip(reason="HIP runtime capture limit: opt in with FTAR_RUN_CAPTURE_LIMITS=1 "
                                   "(the child process crashes in hipStreamEndCapture)")
    for item in items:
        if "capture_runtime_limit" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle():
    """ctypes handle on oracle/liboracle.so (built here if missing)."""
    import oracle_lib
    return oracle_lib.load()
