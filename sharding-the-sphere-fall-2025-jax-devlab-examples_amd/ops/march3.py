"""Pipelined streaming SSP-RK3 step (``ops/csrc/march3_kernel.hip``) of one rank.

The streaming stage (``march_kernel.hip``) is one launch per RK stage: each step
reads and writes the whole state three times.  Here one step is three launches
whose bulk is a single pass over the state:

1. ``march3``: the three stages marched together up every strip of every tile
   (stage s + 1 trails stage s by two rows; rolling rows in registers, the
   conserved stage results in a per-wave LDS ring).  Stage-3 results of the
   cells at least 4 from a tile edge go to the output; the stage-1 / stage-2
   results within ``D`` of a tile edge go to ``pool[1]`` / ``pool[2]`` (stage 1
   also pushes its same-rank ghost copies into ``pool[1]``).
2. the block stage kernel (8x8 blocks) over the blocks along the tile edges:
   stage 2 there (reads ``pool[1]`` with its ghost ring, writes ``pool[2]`` and
   pushes its ghost copies);
3. the same blocks: stage 3 (reads ``pool[2]``, writes the output and pushes the
   output's ghost copies, i.e. the next step's input halo).

The output is a fourth buffer: steps alternate ``pool[0] -> extra -> pool[0]``,
so the native op list covers two steps (period 2).  The reference's time loop
(per RK stage a halo exchange, then the FV kernels; PY:238-246
for the composed exchange) becomes one march per step plus two thin band
launches; the band blocks are the only place the stages meet other tiles.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import native
from ..models.integrators import ssp_rk3

BAND_BLOCK = (8, 8)
M3_COLS = 52          # stage-3 columns per wave (64 lanes - 2 x 2 x 3)
M3_ROWS = (16, 32, 64)


def band_blocks(n: int, T: int, bx: int = 8, by: int = 8) -> Tuple[np.ndarray, int]:
    """Linear ids (t * nby * nbx + yb * nbx + xb, the stage kernel's block
    numbering) of the bx x by blocks holding a cell within 4 of a tile edge,
    and the band depth D: every cell those blocks read (the block plus a ring of
    2) lies within D - 1 of a tile edge."""
    nbx, nby = -(-n // bx), -(-n // by)
    ids, dmax = [], 0
    for yb in range(nby):
        y0, y1 = yb * by, min(n, (yb + 1) * by)
        for xb in range(nbx):
            x0, x1 = xb * bx, min(n, (xb + 1) * bx)
            if x0 < 4 or x1 > n - 4 or y0 < 4 or y1 > n - 4:
                ids.append(yb * nbx + xb)
                xs, ys = np.arange(x0, x1), np.arange(y0, y1)
                dx = np.minimum(xs, n - 1 - xs)
                dy = np.minimum(ys, n - 1 - ys)
                dmax = max(dmax, int(np.minimum(dx[None, :], dy[:, None]).max()))
    per = np.asarray(ids, dtype=np.int64)
    allids = (np.arange(T, dtype=np.int64)[:, None] * (nbx * nby) + per[None, :]).reshape(-1)
    return allids.astype(np.int32), dmax + 3


def march3_unsupported(engine) -> Optional[str]:
    """None if the pipelined step applies to this engine, else the reason."""
    e = engine
    from .hip_compute import HipCompute
    if not isinstance(getattr(e, "compute", None), HipCompute):
        return "needs Engine(backend='hip')"
    if e.compute.phys_id != 2:
        return "shallow water only"
    lim = int(e.physics.kernel_params().get("limiter", 0))
    if lim not in (0, 1, 2, 3):
        return "PLR limiters only (PPM keeps the block kernel)"
    st, ref = e.integ.stages, ssp_rk3().stages
    if len(st) != 3 or any((s.X, s.Q, s.out, s.a0, s.a1, s.a2, s.acc_in, s.acc_out) !=
                           (r.X, r.Q, r.out, r.a0, r.a1, r.a2, r.acc_in, r.acc_out) for s, r in zip(st, ref)):
        return "SSP-RK3 only"
    p = e.plan
    if p.num_recv or p.num_send:
        return "one rank (no remote ghosts)"
    if p.ng != 2:
        return "halo width 2 (PLR)"
    if p.n < 24:
        return "tiles of at least 24 cells"
    _, D = band_blocks(p.n, p.T, *BAND_BLOCK)
    if D > 48 or 2 * D > p.n:
        return "tile too small for the band"
    return None


# The automatic runtime choice keeps the three-launch streaming stage: the
# pipelined step measured even with it at C720 on one MI355X (fp64 405 vs 394
# us/step, fp32 207 vs 181-188: profiles/r6_march3/README.md), so `auto` leaves
# it off and `on` selects it.
MARCH3_AUTO = False


def march3_wanted(engine) -> bool:
    """The size rule of the streaming stage (HipCompute.march_wanted) on a rank
    the pipelined step applies to, when the automatic choice takes it."""
    hc = getattr(engine, "compute", None)
    return MARCH3_AUTO and bool(getattr(hc, "march_wanted", False)) and march3_unsupported(engine) is None


class March3Step:
    """Descriptors of the pipelined step for ``NativeStepper(march3=...)``:
    ``ops()`` returns the native op list of two steps (pool[0] -> extra ->
    pool[0]).  ``rows``: stage-3 rows per wave (16, 32, 64)."""

    def __init__(self, engine, rows: int = 32):
        why = march3_unsupported(engine)
        if why:
            raise ValueError(f"pipelined march step: {why}")
        if rows not in M3_ROWS:
            raise ValueError(f"rows per wave must be one of {M3_ROWS}")
        e = self.e = engine
        hc = e.compute
        self.rows = rows
        p = e.plan
        self.extra = torch.zeros_like(e.pool[0])
        ids, self.D = band_blocks(p.n, p.T, *BAND_BLOCK)
        self.band = torch.as_tensor(ids, device=e.device)
        nb = -(-p.n // BAND_BLOCK[0]) * -(-p.n // BAND_BLOCK[1]) * p.T
        assert ids.size and int(ids.max()) < nb and int(ids.min()) >= 0
        assert len(set(ids.tolist())) == ids.size
        self.ncs = -(-(p.n - 8) // M3_COLS)
        self.nrs = -(-(p.n - 8) // rows)
        self._mdescs: List[native.March3Desc] = []
        self._descs = []

    def _m3desc(self) -> native.March3Desc:
        e = self.e
        st = e.integ.stages
        m = native.March3Desc()
        m.q1 = native.ptr(e.pool[1])
        m.q2 = native.ptr(e.pool[2])
        for k in range(3):
            m.b0[k], m.b1[k], m.b2[k] = st[k].a0, st[k].a1, st[k].a2
        m.D = self.D
        self._mdescs.append(m)
        return m

    def step_descs(self, src: torch.Tensor, dst: torch.Tensor):
        """(march StageDesc, March3Desc, [band stage-2 desc, band stage-3 desc])
        of one step from ``src`` to ``dst``."""
        e = self.e
        hc = e.compute
        st = e.integ.stages
        d = hc.desc(st[0], e.dt, None, 0)
        d.Q = d.X = native.ptr(src)
        d.out = native.ptr(dst)
        m = self._m3desc()
        band = []
        for s in (st[1], st[2]):
            bd = hc.desc(s, e.dt, self.band, self.band.numel())
            bd.X = native.ptr(src)
            if s.out == 0:
                bd.out = native.ptr(dst)
            band.append(bd)
        self._descs.append((d, m, band))
        return d, m, band

    def ops(self):
        from .native_runtime import OP_MARCH3, OP_STAGE, StspOp
        e = self.e
        hc = e.compute
        out = []
        for src, dst in ((e.pool[0], self.extra), (self.extra, e.pool[0])):
            d, m, band = self.step_descs(src, dst)
            op = StspOp()
            op.type = OP_MARCH3
            op.dtype = hc.dcode
            op.phys = hc.phys_id
            op.by = self.rows
            op.stage = d
            op.fused = ctypes.addressof(m)
            out.append(op)
            for bd in band:
                op = StspOp()
                op.type = OP_STAGE
                op.phys, op.dtype = hc.phys_id, hc.dcode
                op.bx, op.by = BAND_BLOCK
                op.stage = bd
                out.append(op)
        return out

    def launch_step(self, src: torch.Tensor, dst: torch.Tensor, stream: Optional[int] = None) -> None:
        """One pipelined step from ``src`` to ``dst`` issued directly (tests)."""
        e = self.e
        hc = e.compute
        L = native.require_native()
        s = native.current_stream_handle() if stream is None else stream
        d, m, band = self.step_descs(src, dst)
        native.check(L.stsp_march3_launch(hc.dcode, self.rows, ctypes.byref(d), ctypes.byref(m), s), "march3")
        for bd in band:
            native.check(L.stsp_stage_launch(hc.phys_id, hc.dcode, BAND_BLOCK[0], BAND_BLOCK[1], ctypes.byref(bd), s),
                         "band stage")
        self._descs.clear()
        self._mdescs.clear()

    def step(self, nsteps: int = 1) -> None:
        """nsteps pipelined steps of the engine's state (eager, tests)."""
        e = self.e
        for _ in range(nsteps):
            self.launch_step(e.pool[0], self.extra)
            e.pool[0], self.extra = self.extra, e.pool[0]
            e.time += e.dt
            e.step_count += 1
