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


_LIB = []


def _lib():
    if not _LIB:
        L = None
        if torch.cuda.is_available():
            try:
                from ..ops import native
                L = native.load(build_if_missing=False)
                L = L if hasattr(L, "stsp_roctx_push") else None
            except Exception:
                L = None
        _LIB.append(L)
    return _LIB[0]


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


class PhaseTimes:
    """Host wall time accumulated per named phase; every phase is also a
    roctx range, so ``rocprofv3 --marker-trace`` shows the driver's step /
    history / checkpoint / metrics phases next to the kernels.

        ph = PhaseTimes()
        with ph("step"): ...
        ph.times -> {"step": seconds, ...}
    """

    def __init__(self):
        self.times: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}

    @contextlib.contextmanager
    def __call__(self, name: str):
        t0 = time.perf_counter()
        with trace_range(name):
            try:
                yield
            finally:
                self.times[name] = self.times.get(name, 0.0) + time.perf_counter() - t0
                self.counts[name] = self.counts.get(name, 0) + 1


def summarize(times: Dict[str, float]) -> str:
    tot = sum(times.values()) or 1.0
    return "\n".join(f"  {k:24s} {v * 1e3:10.3f} ms  {100 * v / tot:5.1f} %" for k, v in
                     sorted(times.items(), key=lambda kv: -kv[1]))
