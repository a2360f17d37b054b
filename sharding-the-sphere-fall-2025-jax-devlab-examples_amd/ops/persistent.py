"""Persistent stepping: many whole time steps in ONE kernel launch
(``ops/csrc/step_kernel.hip``), the MI355X answer to the C96 latency regime.

At C96 one RK stage is ~3 us of dependent work per block, and a
launch-per-stage step pays a dependent kernel boundary (~1.5-1.9 us) plus a
full window / geometry / state reload from memory for each of its 3 stages.
The persistent step kernel keeps each block's state in registers and its
geometry in registers / LDS for the whole launch; a stage boundary is a
granule hand-off of the halo ring between side-neighbouring blocks only
(8-byte {tag, payload} stores into an exchange buffer laid out like the padded
state; the reading thread re-reads until the tag matches), so no block ever
waits on the whole grid and no fence, flag or drain is on the critical path.

Requirements checked here before anything is launched: one rank (no remote
ghosts), an integrator whose stages all combine the step-start state with the
previous stage output (SSP-RK2, SSP-RK3), every block co-resident (occupancy
API bound), and a symmetric block read relation (the two-slot argument in
step_kernel.hip).  Race freedom is argued per neighbour pair, the structural
argument of the reference's "no device appears twice in the same
communication stage" (PDF s.9).
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np
import torch

from . import native
from ..models.integrators import step_kernel_compatible

STEP_SHAPES = ((16, 16), (16, 8), (8, 8))


class StepDesc(ctypes.Structure):
    _fields_ = [
        ("st", native.StageDesc), ("nst", ctypes.c_int), ("nsteps", ctypes.c_int),
        ("a0", ctypes.c_double * 4), ("a1", ctypes.c_double * 4), ("a2", ctypes.c_double * 4),
        ("xb", ctypes.c_void_p), ("epoch", ctypes.c_void_p), ("err", ctypes.c_void_p),
        ("timeout_ticks", ctypes.c_longlong), ("dbg", ctypes.c_void_p),
    ]


def producer_blocks(plan, bx: int, by: int, NG: int) -> np.ndarray:
    """[nblocks, maxnbr] ids of the blocks whose stage output each block's
    window reads; -1 padded.  A window cell is read iff it lies within NG of
    the block's real cells along a row or a column of them (the
    dimension-split stencils; window corners and, for a partial block, the
    rows / columns past the tile edge are never read), exactly the cells the
    step kernel waits for."""
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
                xe, ye = min(x0 + bx, n), min(y0 + by, n)
                cells = {(x, y) for y in range(y0, ye) for x in range(x0 - NG, xe + NG)}
                cells |= {(x, y) for x in range(x0, xe) for y in range(y0 - NG, ye + NG)}
                s = set()
                for x, y in cells:
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


def symmetric(nbr: np.ndarray) -> bool:
    """True if every block that a block reads from also reads from it."""
    sets = [set(int(x) for x in row if x >= 0) for row in nbr]
    return all(b in sets[p] for b, s in enumerate(sets) for p in s)


def _lib():
    L = native.require_native()
    L.stsp_step_launch.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(StepDesc), ctypes.c_void_p]
    L.stsp_step_launch.restype = ctypes.c_int
    L.stsp_step_max_blocks.argtypes = [ctypes.c_int] * 5
    L.stsp_step_max_blocks.restype = ctypes.c_int
    return L


class PersistentStepper:
    """``run(nsteps)``: nsteps whole steps of an ``Engine(backend='hip')`` in
    ceil(nsteps / max_steps_per_launch) launches of the persistent step kernel.
    Bitwise equal to launch-per-stage stepping."""

    def __init__(self, engine, timeout_s: float = 2.0, max_steps_per_launch: int = 1000, block=None,
                 exchange: str = "uncached"):
        from .hip_compute import HipCompute
        e = engine
        if not isinstance(e.compute, HipCompute):
            raise RuntimeError("PersistentStepper needs an Engine with backend='hip'")
        hc = e.compute
        if hc.remote or e.plan.num_recv or e.plan.num_send:
            raise RuntimeError("persistent stepping is single-rank (no remote halos)")
        if not step_kernel_compatible(e.integ):
            raise RuntimeError(f"integrator {e.integ.name}: the step kernel needs stages that combine the "
                               "step-start state with the previous stage output (SSP-RK2 / SSP-RK3)")
        want = tuple(block) if block is not None else (hc.bx, hc.by)
        if want not in STEP_SHAPES:
            want = (16, 16)
        if (hc.bx, hc.by) != want:
            e.block = want
            e.compute = hc = HipCompute(e)
        self.e = e
        self.L = _lib()
        lim = int(e.physics.kernel_params().get("limiter", 0))
        if lim == 4:
            # measured on MI355X (round 2): the PPM instantiation differs from
            # launch-per-stage stepping after a few launches; until that is
            # understood the persistent path is PLR-only
            raise NotImplementedError("persistent stepping supports PLR limiters only (not PPM)")
        if hc.phys_id != 1:
            # the panel-edge ghost interpolation (models/base.py::reconstruct,
            # stage_kernel.hip phase 1a) reads strip cells beyond a block's rows,
            # which the persistent kernel's side-neighbour granule hand-off does
            # not deliver; it lost to graph replay anyway (profiles/r2_persistent)
            raise NotImplementedError("persistent stepping predates the panel-edge reconstruction: "
                                      "diffusion only")
        maxb = self.L.stsp_step_max_blocks(hc.phys_id, hc.dcode, hc.bx, hc.by, lim)
        if maxb <= 0:
            raise RuntimeError(f"step kernel not available for this configuration ({maxb})")
        if hc.nblocks > maxb:
            raise RuntimeError(f"{hc.nblocks} blocks exceed the {maxb} co-resident blocks of this GPU")
        nb = producer_blocks(e.plan, hc.bx, hc.by, e.physics.halo)
        if not symmetric(nb):
            raise RuntimeError("block read relation is not symmetric: two exchange slots are not enough")
        F, S = e.physics.F, e.plan.S
        G = torch.tensor([], dtype=e.dtype).element_size() // 4
        if 2 * S * F * G * 8 >= 2 ** 31:
            raise RuntimeError("grid too large for the step kernel's 32-bit exchange offsets")
        dev = e.device
        # Exchange buffer.  "uncached" (default): hipExtMallocWithFlags(
        # hipDeviceMallocUncached), every granule store and poll goes to memory,
        # never to a stale cache line.  Measured (tools/persist_stamps.py,
        # profiles/r2_persist_stamps_*.json): with a cached (hipMalloc / torch)
        # buffer the agent-scope polls saw a new granule only ~10-20 us after it
        # was stored, so every stage waited ~12 us for its halo.
        self.exchange = exchange
        self._xb_raw = None
        nbytes = 2 * S * F * G * 8
        if exchange in ("uncached", "finegrained"):
            from .xgmi import _declare as _xg_declare
            _xg_declare(self.L)
            self.L.stsp_alloc_flags.argtypes = [ctypes.c_size_t, ctypes.c_uint, ctypes.POINTER(ctypes.c_void_p)]
            self.L.stsp_alloc_flags.restype = ctypes.c_int
            raw = ctypes.c_void_p()
            rc = self.L.stsp_alloc_flags(ctypes.c_size_t(nbytes), 3 if exchange == "uncached" else 1,
                                         ctypes.byref(raw))
            if rc != 0:
                raise RuntimeError(f"uncached exchange buffer allocation failed ({rc})")
            self._xb_raw = raw.value
            self.xb = None
        else:
            self.xb = torch.zeros(2 * S * F * G, dtype=torch.int64, device=dev)
        self.epoch = torch.zeros(hc.nblocks, dtype=torch.int32, device=dev)
        self.err = torch.zeros(4, dtype=torch.int32, device=dev)
        self.timeout_ticks = int(timeout_s * 1e8)
        self.max_steps = max(1, int(max_steps_per_launch))
        import os
        self.dbg = (torch.zeros(4096 + hc.nblocks * 128, dtype=torch.int64, device=dev)
                    if os.environ.get("STSP_VARIANT", "").startswith("stepdbg") else None)
        self.stats = {"persistent_steps": 0, "launches": 0, "eager_steps": 0, "graph_steps": 0}
        self._build()

    def _build(self):
        e, hc = self.e, self.e.compute
        st0 = e.integ.stages[0]
        d = StepDesc()
        d.st = hc.desc(st0, e.dt, None, hc.nblocks)
        d.st.X = d.st.Q = d.st.out = native.ptr(e.pool[0])   # the state: read at the start, written at the end
        d.st.acc_in = d.st.acc_out = 0
        d.nst = len(e.integ.stages)
        for k, st in enumerate(e.integ.stages):
            d.a0[k], d.a1[k], d.a2[k] = st.a0, st.a1, st.a2
        d.xb = self._xb_raw if self._xb_raw is not None else native.ptr(self.xb)
        d.epoch = native.ptr(self.epoch)
        d.err = native.ptr(self.err)
        d.timeout_ticks = self.timeout_ticks
        d.dbg = native.ptr(self.dbg) if self.dbg is not None else 0
        self._d = d

    def set_dt(self, dt: float) -> None:
        self.e.dt = dt
        self._build()

    def _launch(self, k: int) -> None:
        hc = self.e.compute
        self._d.nsteps = k
        rc = self.L.stsp_step_launch(hc.phys_id, hc.dcode, hc.bx, hc.by, ctypes.byref(self._d),
                                     native.current_stream_handle())
        native.check(rc, "persistent step launch")
        self.stats["launches"] += 1

    def run(self, nsteps: int) -> None:
        e = self.e
        left = nsteps
        while left > 0:
            k = min(left, self.max_steps)
            if k * len(e.integ.stages) < 2:     # one single-stage step: launch-per-stage
                e.step(k)
                self.stats["eager_steps"] += k
            else:
                self._launch(k)
                self.stats["persistent_steps"] += k
                e.time += k * e.dt
                e.step_count += k
            left -= k

    def check(self) -> None:
        """Raise if a hand-off timed out (synchronises)."""
        if int(self.err[0].item()) != 0:
            raise RuntimeError("persistent step kernel: a halo hand-off timed out (state invalid)")

    def close(self) -> None:
        if getattr(self, "_xb_raw", None):
            torch.cuda.synchronize(self.e.device)
            self.L.stsp_xg_free(ctypes.c_void_p(self._xb_raw))
            self._xb_raw = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
