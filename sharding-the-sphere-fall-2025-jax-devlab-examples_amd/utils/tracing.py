"""Tracing / profiling hooks (the reference has none).

* ``trace_range(name)``: a roctx range (rocprofiler-sdk-roctx, recorded by
  ``rocprofv3 --marker-trace``) around any host region; no-op without a GPU.
* ``Timer``: host wall time plus HIP-event device time for a region.
* The native runtime emits roctx ranges per op when created with roctx=True.

Kernel-level evidence is collected with rocprofv3 (see tools/*.sh):
``rocprofv3 --kernel-trace --stats`` for per-kernel time and ``--pmc`` for
counters (in separate runs).  The reference's only performance artefact is
the analytic roofline of PDF s.19 (utils/roofline.py).
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, Optional

import torch


def _lib():
    if not torch.cuda.is_available():
        return None
    try:
        from ..ops import native
        L = native.load(build_if_missing=False)
        return L if hasattr(L, "stsp_roctx_push") else None
    except Exception:
        return None


@contextlib.contextmanager
def trace_range(name: str):
    L = _lib()
    if L is not None:
        import ctypes
        L.stsp_roctx_push.argtypes = [ctypes.c_char_p]
        L.stsp_roctx_push(name.encode())
    try:
        yield
    finally:
        if L is not None:
            L.stsp_roctx_pop()


class Timer:
    """with Timer() as t: ...;  t.wall_s, t.device_ms"""

    def __init__(self, device: Optional[torch.device] = None):
        self.device = device
        self.wall_s = 0.0
        self.device_ms: Optional[float] = None

    def __enter__(self):
        self._cuda = torch.cuda.is_available() and (self.device is None or torch.device(self.device).type == "cuda")
        if self._cuda:
            self._e0 = torch.cuda.Event(enable_timing=True)
            self._e1 = torch.cuda.Event(enable_timing=True)
            self._e0.record()
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self._cuda:
            self._e1.record()
            torch.cuda.synchronize()
            self.device_ms = self._e0.elapsed_time(self._e1)
        self.wall_s = time.perf_counter() - self._t0
        return False


def summarize(times: Dict[str, float]) -> str:
    tot = sum(times.values()) or 1.0
    return "\n".join(f"  {k:24s} {v * 1e3:10.3f} ms  {100 * v / tot:5.1f} %" for k, v in
                     sorted(times.items(), key=lambda kv: -kv[1]))
