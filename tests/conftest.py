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


@pytest.fixture(autouse=True)
def _heap_canary(request):
    """STSP_HEAP_CANARY=1 (GPU runs): after every GPU test, collect garbage
    (so destructors run here, not inside a later test) and check that fresh
    device allocations do not overlap (each filled with its own value and
    read back) and that a session-long canary buffer is unchanged."""
    yield
    if os.environ.get("STSP_HEAP_CANARY") != "1" or "gpu" not in request.keywords:
        return
    import gc
    import torch
    if not torch.cuda.is_available():
        return
    gc.collect()
    torch.cuda.synchronize()
    if not hasattr(_heap_canary, "keep"):
        _heap_canary.keep = torch.full((1 << 23,), 7.0, dtype=torch.float64, device="cuda")
    bad_keep = int((_heap_canary.keep != 7.0).sum())
    xs = [torch.full(((1 << (8 + k % 14)) + 8 * k,), float(k), dtype=torch.float64, device="cuda")
          for k in range(96)]
    bad = [k for k, x in enumerate(xs) if not bool((x == float(k)).all())]
    print(f"\n[heap-canary] after {request.node.nodeid}: keep bad {bad_keep}, overlapping {bad[:8]}",
          flush=True)
    del xs



@pytest.fixture(autouse=True)
def _ring_guard(request):
    """STSP_RING_GUARD=1 (GPU runs): every xGMI ring carries 64 KiB guard
    regions on both sides (ops/csrc/runtime.cpp); after every GPU test they
    are checked, and a store past either end of a ring fails the test that
    made it (the round-4 post-free corruption hunt, profiles/r4_ring)."""
    yield
    if os.environ.get("STSP_RING_GUARD") != "1" or "gpu" not in request.keywords:
        return
    import torch
    if not torch.cuda.is_available():
        return
    from stsphere.ops import native
    L = native.require_native()
    import ctypes
    L.stsp_xg_check_guards.restype = ctypes.c_longlong
    torch.cuda.synchronize()
    bad = int(L.stsp_xg_check_guards())
    print(f"\n[ring-guard] after {request.node.nodeid}: {bad} guard words changed", flush=True)
    assert bad == 0, f"{bad} guard words around the xGMI rings changed (a store past a ring's end)"
