import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
# XDDP_PKG_ROOT: import the package from another root (the sanitizer builds' package copies,
# tests/test_sanitizers_cpu.py); spawned ranks inherit this sys.path
_root = os.environ.get("XDDP_PKG_ROOT")
if _root:
    sys.path.insert(0, _root)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
# flight-record dumps from intentionally failing collectives go to a private temp dir
import tempfile  # noqa: E402

os.environ.setdefault("XDDP_FLIGHT_DUMP_PREFIX", os.path.join(tempfile.mkdtemp(prefix="xddp_flight_"), "rank_"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
