"""Persistent multi-step stepping for small grids (the C96 latency regime).

At C96 a single 16x16-cell block of the fused stage kernel takes ~5.6 us per
launch against a ~1.6 us empty-kernel floor (measured, tools/kprobe.py
--limit 1), i.e. the per-launch critical path (cold instruction cache, kernel
arguments, dependent memory round trips) dominates, not bandwidth.
``PersistentStepper`` launches ONE cooperative kernel for many steps: each
workgroup keeps its block for every stage, and a stage boundary is a
neighbour-only hand-off (sc1 write-through stores + per-block epoch flag,
bounded polls) instead of a kernel boundary.  Single rank, SSP-RK3 (the
stage/buffer sequence must be race-free with neighbours one stage apart,
``integrators.persistent_safe``).  Race freedom is argued per neighbour pair,
the same structural argument as the reference's "no device appears twice in
the same communication stage" (PDF s.9).
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np
import torch

from . import native
from ..models.integrators import persistent_safe


def producer_blocks(plan, bx: int, by: int, NG: int) -> np.ndarray:
    """[nblocks, maxnbr] ids of the blocks whose stage output each block's
    window (block + NG halo, corners excluded) reads; -1 padded."""
    L = plan.layout
    n, T = plan.n, plan.T
    nbx, nby = -(-n // bx), -(-n // by)
    src = L.ghost_sources(plan.rank)        # [T,4,ng,n] global cells
    tid_of = {t: li for li, t in enumerate(plan.tiles)}

    def block_of(li, i, j):
        return (li * nby + j // by) * nbx + i // bx

    out: List[set] = []
    for li in range(T):
        for yb in range(nby):
            for xb in range(nbx):
                me = (li * nby + yb) * nbx + xb
                x0, y0 = xb * bx, yb * by
                s = set()
                for y in range(y0 - NG, min(n + NG, y0 + by + NG)):
                    for x in range(x0 - NG, min(n + NG, x0 + bx + NG)):
                        if (x < x0 or x >= x0 + bx) and (y < y0 or y >= y0 + by):
                            continue        # window corners: loaded, never used by the stencils
                        ox, oy = x < 0 or x >= n, y < 0 or y >= n
                        if ox and oy:
                            continue
                        if not ox and not oy:
                            s.add(block_of(li, x, y))
                            continue
                        if x < 0:
                            side, layer, pos = 0, -1 - x, y
                        elif x >= n:
                            side, layer, pos = 1, x - n, y
                        elif y < 0:
                            side, layer, pos = 2, -1 - y, x
                        else:
                            side, layer, pos = 3, y - n, x
                        g = int(src[li, side, layer, pos])
                        t2, i2, j2 = L.locate(np.array([g]))
                        s.add(block_of(tid_of[int(t2[0])], int(i2[0]), int(j2[0])))
                s.discard(me)
                out.append(s)
    m = max(1, max(len(s) for s in out))
    arr = np.full((len(out), m), -1, dtype=np.int32)
    for b, s in enumerate(out):
        arr[b, :len(s)] = sorted(s)
    return arr


class PersistentStepper:
    BX = BY = 16

    def __init__(self, engine, timeout_s: float = 2.0, max_steps_per_launch: int = 1000):
        from .hip_compute import HipCompute
        e = engine
        if not isinstance(e.compute, HipCompute):
            raise RuntimeError("PersistentStepper needs an Engine with backend='hip'")
        hc = e.compute
        if hc.remote:
            raise RuntimeError("persistent stepping is single-rank (no remote halos)")
        if (hc.bx, hc.by) != (self.BX, self.BY):
            if e.block is not None:
                raise RuntimeError("persistent stepping uses 16x16 blocks")
            # the engine picked a smaller block for a small grid: rebuild its
            # stage tables for the persistent kernel's fixed 16x16 shape
            e.block = (self.BX, self.BY)
            e.compute = hc = HipCompute(e)
        if not persistent_safe(e.integ):
            raise RuntimeError(f"integrator {e.integ.name} is not race-free with a one-stage neighbour lag")
        props = torch.cuda.get_device_properties(e.device)
        if hc.nblocks > props.multi_processor_count:
            raise RuntimeError(f"{hc.nblocks} blocks exceed {props.multi_processor_count} CUs (one block per CU)")
        self.e = e
        self.L = native.require_native()
        self.L.stsp_persistent_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                                      ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p]
        self.L.stsp_persistent_launch.restype = ctypes.c_int
        nb = producer_blocks(e.plan, self.BX, self.BY, e.physics.halo)
        assert nb.shape[0] == hc.nblocks and nb.max() < hc.nblocks
        self.maxnbr = nb.shape[1]
        self.nbr = torch.as_tensor(nb, device=e.device)
        self.flags = torch.zeros(((hc.nblocks + 3) // 4) * 4, dtype=torch.int32, device=e.device)
        self.err = torch.zeros(4, dtype=torch.int32, device=e.device)
        self.timeout_s = timeout_s
        self.max_steps = max_steps_per_launch
        self._build()

    def _build(self):
        e, hc = self.e, self.e.compute
        ds = [hc.desc(st, e.dt, None, hc.nblocks) for st in e.integ.stages]
        self._descs = (native.StageDesc * len(ds))(*ds)

    def set_dt(self, dt):
        self.e.dt = dt
        self._build()

    def run(self, nsteps: int) -> None:
        e, hc = self.e, self.e.compute
        left = nsteps
        while left > 0:
            k = min(left, self.max_steps)
            rc = self.L.stsp_persistent_launch(hc.phys_id, hc.dcode, self.BX, self.BY, self._descs,
                                               len(self._descs), k, native.ptr(self.flags), native.ptr(self.nbr),
                                               self.maxnbr, native.ptr(self.err), self.timeout_s,
                                               native.current_stream_handle())
            native.check(rc, "persistent launch")
            left -= k
        e.time += nsteps * e.dt
        e.step_count += nsteps

    def check(self) -> None:
        """Raise if any launch timed out (synchronises)."""
        if int(self.err[0].item()) != 0:
            raise RuntimeError("persistent kernel: neighbour hand-off timed out (state invalid)")
