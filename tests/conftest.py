import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    # xdist workers share the CPUs: keep torch's intra-op pool to a fair share
    # (oversubscribed pools made the numerics tests 20x slower)
    nw = os.environ.get("PYTEST_XDIST_WORKER_COUNT")
    if nw:
        import torch
        torch.set_num_threads(max(1, (os.cpu_count() or 8) // int(nw)))
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native library")
    config.addinivalue_line("markers", "slow: long-running numerics test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
