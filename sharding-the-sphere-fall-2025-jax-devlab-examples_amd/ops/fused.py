"""Fused time step (temporal blocking): one launch per SSP-RK step.

The launch-per-stage path (``stage_kernel.hip``) pays a dependent kernel
boundary and a window round trip per RK stage, three per SSP-RK3 step.  The
reference composes its whole halo exchange into one compiled program for the
same reason (PY:238-246; PDF s.10 "Why two JITs?").  Here a whole step is one
launch: every block loads its ``B x B`` cells plus a ring ``R = ns * 2`` wide
(``ns`` stages, PLR reads 2 cells per stage), then advances the ring through
the earlier stages by redundant recompute, so no block waits for another
inside the step.

Ring cells beyond a cube edge belong to another panel.  They are updated in
their own panel's frame, exactly as that panel's own tile computes them in the
stage-by-stage scheme (models/base.py::reconstruct):

* a cell next to a panel edge reads its neighbour across the edge as the
  other panel's edge cells **interpolated onto its own grid line** (the
  Putman-Lin ghost, ``panel_edge_tables``).  Those values live in per-block
  *ghost strips* keyed by (reader region, side, along-edge position); the
  table entry names the two window cells and the weight;
* at a cube corner the window's diagonal quadrant has no cells.  The faces of
  the panel-edge cells that point into it are the third cube edge; they are
  listed as *corner faces* (cell, side, partner cell, partner side) and get
  the flux computed from both panels' reconstructions, as FV3's direction-split
  corner fill does.

Everything the kernel needs beyond the state is precomputed here, on the host,
from the same tables the oracle uses (ghost sources, ``pe_base`` / ``pe_t``,
the edge normals and lengths), so the fused step reproduces the stage-by-stage
step to rounding.  ``fused_step_torch`` is the PyTorch rendering of the kernel
(same tables, same phases) and is checked against ``Engine.step`` on CPU;
``ops/csrc/fused_step.hip`` is the gfx950 kernel.

Window coordinates: cell ``(u, v)``, ``u`` along x (columns), ``v`` along y
(rows), ``u, v in [0, W)``, ``W = B + 2 R``; panel coordinates
``(X0 + u, Y0 + v)`` in the block's panel (outside ``[0, N)`` = another panel).
Stage ``s`` (1-based) updates the square ``[lo_s, hi_s)`` with
``lo_s = R - 2 (ns - s)``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..models.base import panel_edge_tables
from ..parallel.layout import TileLayout, ghost_xy
from ..parallel.topology import neighbor_cells


def native_stream(device) -> int:
    from .native import current_stream_handle
    return current_stream_handle(device)

REG_P, REG_W, REG_E, REG_S, REG_N = 0, 1, 2, 3, 4
NREG = 5
# window sides: 0 = -x, 1 = +x, 2 = -y, 3 = +y
SIDE_VEC = ((-1, 0), (1, 0), (0, -1), (0, 1))
NG_PLR = 2


def region(X, Y, N):
    """Region code of extended-panel coordinates: P inside, W/E/S/N across one
    panel edge, -1 beyond a cube corner (no cell)."""
    X = np.asarray(X)
    Y = np.asarray(Y)
    inx = (X >= 0) & (X < N)
    iny = (Y >= 0) & (Y < N)
    r = np.full(np.broadcast(X, Y).shape, -1, dtype=np.int64)
    r[inx & iny] = REG_P
    r[(X < 0) & iny] = REG_W
    r[(X >= N) & iny] = REG_E
    r[(Y < 0) & inx] = REG_S
    r[(Y >= N) & inx] = REG_N
    return r


def _region_point(N: int, reg: int) -> Tuple[int, int]:
    h = N // 2
    return {REG_P: (h, h), REG_W: (-2, h), REG_E: (N, h), REG_S: (h, -2)}.get(reg, (h, N))


def frame_map(N: int, face: int, reg: int) -> Tuple[int, np.ndarray]:
    """(panel of region ``reg`` around ``face``, 2x2 integer matrix M) with
    M @ (du, dv) = the step in that panel's own (i, j) index frame for a step
    (du, dv) in ``face``'s extended index frame."""
    p = _region_point(N, reg)
    X = np.array([p[0], p[0] + 1, p[0]])
    Y = np.array([p[1], p[1], p[1] + 1])
    F, I, J = neighbor_cells(N, face, X, Y)
    assert F[0] == F[1] == F[2] >= 0
    M = np.array([[I[1] - I[0], I[2] - I[0]], [J[1] - J[0], J[2] - J[0]]], dtype=np.int64)
    return int(F[0]), M


def frame_code(face: int) -> int:
    """Panel frame for the kernel's to_global: axis of e_i (bits 0-1), of e_j
    (bits 2-3), sign bits of e_i, e_j, n (6, 7, 8); FACE_FRAMES rows are n, e_i, e_j."""
    from ..parallel.topology import FACE_FRAMES
    n, ei, ej = FACE_FRAMES[face]
    ax = lambda v: int(np.argmax(np.abs(v)))
    neg = lambda v: int(v[ax(v)] < 0)
    assert len({ax(n), ax(ei), ax(ej)}) == 3
    return ax(ei) | (ax(ej) << 2) | (neg(ei) << 6) | (neg(ej) << 7) | (neg(n) << 8)


def kernel_geometry(layout: TileLayout, grid) -> Dict[str, np.ndarray]:
    """Panel-independent geometry the gfx950 kernel reads instead of per-cell
    records (fused_step.hip, prologue; the window cell's panel index comes from
    the cube topology, window_cell):

      frames [6] int32        frame_code per panel
      tane [N+1]              tan of the grid-line angles
      crec [N*N, 8]           by panel-local index (equal on every panel): 1/A, the
                              curvature sum S = sum(L m) over the cell's faces and the
                              cell centre, both in panel-local components (e_i, e_j, n), 0
      lxt  [N, N+1]           x-edge lengths (j, i'); y-edge (j', i) = lxt[i, j']
    """
    N = layout.N
    lx, ly = grid.x_edge_lengths(), grid.y_edge_lengths()
    mx, my = grid.x_edge_normals(), grid.y_edge_normals()
    # panel 4 has the identity frame (n, e_i, e_j) = (x, y, z): local = (y, z, x)
    f4 = 4
    Sv = (lx[f4, :, 1:, None] * mx[f4, None, 1:, :] - lx[f4, :, :-1, None] * mx[f4, None, :-1, :]
          + ly[f4, 1:, :, None] * my[f4, 1:, None, :] - ly[f4, :-1, :, None] * my[f4, :-1, None, :])   # [N,N,3]
    c4 = grid.centers()[f4]                                   # [N, N, 3] (x, y, z) = (n, e_i, e_j)
    crec = np.zeros((N * N, 8))
    crec[:, 0] = (1.0 / grid.areas()[0]).ravel()
    crec[:, 1], crec[:, 2], crec[:, 3] = Sv[..., 1].ravel(), Sv[..., 2].ravel(), Sv[..., 0].ravel()
    crec[:, 4], crec[:, 5], crec[:, 6] = c4[..., 1].ravel(), c4[..., 2].ravel(), c4[..., 0].ravel()
    return {
        "frames": np.array([frame_code(f) for f in range(6)], dtype=np.int32),
        "tane": np.tan(grid.alpha_edges()), "crec": crec, "lxt": lx[0].copy(),
    }


def _side_of(di: int, dj: int) -> int:
    """Tile side index (0 W, 1 E, 2 S, 3 N) of an index-frame unit step."""
    return {(-1, 0): 0, (1, 0): 1, (0, -1): 2, (0, 1): 3}[(int(di), int(dj))]


@dataclass
class FusedDims:
    B: int
    ns: int
    R: int
    W: int
    L1: int      # first window row/column updated by stage 1
    H1: int      # cells per row updated by stage 1

    @classmethod
    def make(cls, B: int, ns: int) -> "FusedDims":
        R = NG_PLR * ns
        W = B + 2 * R
        L1 = R - NG_PLR * (ns - 1)
        H1 = B + 2 * NG_PLR * (ns - 1)
        return cls(B, ns, R, W, L1, H1)

    def stage_range(self, s: int) -> Tuple[int, int]:
        """[lo, hi) of window rows/columns that stage s (1-based) updates."""
        lo = self.R - NG_PLR * (self.ns - s)
        return lo, self.W - lo

    @property
    def nfx(self) -> int:        # x-faces of the stage-1 set: rows H1, lines H1+1
        return self.H1 * (self.H1 + 1)


class FusedPlan:
    """Per-block tables of the fused step for one rank (numpy; see module doc).

    Arrays (nb = number of blocks, bid = (tile_local * nby + yb) * nbx + xb):
      org   [nb, 4]  int32  X0, Y0 (panel coords of the window origin), tile_local, 0
      src   [nb, W*W] int32 padded state offset of each window cell's source
                            cell; -1 beyond a cube corner; <= -2: receive slot -2-src
      reg   [nb, W*W] int8  region code (P W E S N, -1 none)
      nrm   [nb, 2, 5, W+1, 3] float64  unit normal of grid line k (between
                            columns / rows k-1 and k) of each region, oriented +u / +v
      lx    [nb, H1, H1+1]  float64  length of x-face (row L1+r, line L1+c)
      ly    [nb, H1+1, H1]  float64  length of y-face (line L1+r, column L1+c)
      gtab  [nb, G, 4] int32 (strip = reg*4+side, pos, slot0, slot1), gt [nb, G] weights,
            gcnt [nb]
      ctab  [nb, C, 6] int32 (slot_c, side_c, slot_d, side_d, fslot_c, fslot_d),
            cgeo [nb, C, 4] (normal out of c, length), ccnt [nb]
    Face slots (fslot) index the stage-1 flux arrays: x-face (r, c) -> r (H1+1) + c,
    y-face (r, c) -> H1 (H1+1) + r H1 + c; -1 = outside them.
    """

    def __init__(self, layout: TileLayout, rank: int, grid, B: int = 16, ns: int = 3,
                 source=None, other_tiles_remote: bool = False):
        self.layout = layout
        self.rank = rank
        self.grid = grid
        N, n, t = layout.N, layout.n, layout.t
        if n % B:
            raise ValueError(f"fused step: tile size {n} is not a multiple of the block size {B}")
        d = FusedDims.make(B, ns)
        if d.R >= N:
            raise ValueError(f"fused step: ring width {d.R} needs C{N} > {d.R}")
        self.d = d
        self.N, self.n, self.B, self.ns = N, n, B, ns
        plan = layout.plan(rank)
        self.tiles = list(plan.tiles)
        self.T = len(self.tiles)
        self.nbx = self.nby = n // B
        self.nb = self.T * self.nbx * self.nby
        # where a global cell lives: padded local offset (>= 0) or receive code;
        # other_tiles_remote (loopback rehearsal): a block reads every cell of
        # another tile as a remote cell (-2), through the rank's own ring
        self._source = source or (lambda g: layout.local_flat(g))
        self._other_remote = other_tiles_remote
        self._lx = grid.x_edge_lengths()
        self._ly = grid.y_edge_lengths()
        self._mx = grid.x_edge_normals()
        self._my = grid.y_edge_normals()
        self._pe_cache: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
        self._build()

    # ---- helpers -----------------------------------------------------------
    def _pe(self, tid: int):
        if tid not in self._pe_cache:
            b, t = panel_edge_tables(self.N, self.layout, [tid], 1)
            self._pe_cache[tid] = (b[0, :, 0], t[0, :, 0])
        return self._pe_cache[tid]

    def _ghost_source(self, tid: int, side: int, pos: int) -> int:
        """Global flat id of layer-0 ghost ``pos`` of tile ``tid``'s ``side``."""
        L = self.layout
        f, I0, J0 = L.tile_origin(tid)
        x, y = ghost_xy(side, 0, np.array([pos]), self.n)
        F, I, J = neighbor_cells(self.N, f, I0 + x, J0 + y)
        assert F[0] >= 0
        return int(L.global_flat(F[0], I[0], J[0]))

    def _face_normal(self, face, i, j, di, dj, plus: bool) -> np.ndarray:
        """Unit normal pointing along index step (di, dj) of the face on the
        (di, dj) side of cell (i, j) if plus, else on the -(di, dj) side."""
        if plus:
            if di == 1:
                return self._mx[face, i + 1]
            if di == -1:
                return -self._mx[face, i]
            if dj == 1:
                return self._my[face, j + 1]
            return -self._my[face, j]
        # face on the -(di, dj) side, normal still along +(di, dj)
        if di == 1:
            return self._mx[face, i]
        if di == -1:
            return -self._mx[face, i + 1]
        if dj == 1:
            return self._my[face, j]
        return -self._my[face, j + 1]

    def _face_length(self, face, i, j, di, dj, plus: bool) -> float:
        if not plus:
            di, dj = -di, -dj
        if di == 1:
            return float(self._lx[face, j, i + 1])
        if di == -1:
            return float(self._lx[face, j, i])
        if dj == 1:
            return float(self._ly[face, j + 1, i])
        return float(self._ly[face, j, i])

    def fslot(self, u: int, v: int, side: int) -> int:
        """Stage-1 flux-array slot of the face on ``side`` of window cell (u, v)."""
        d = self.d
        L1, H1 = d.L1, d.H1
        if side in (0, 1):
            k = u + (side == 1)
            r, c = v - L1, k - L1
            if 0 <= r < H1 and 0 <= c <= H1:
                return r * (H1 + 1) + c
            return -1
        k = v + (side == 3)
        r, c = k - L1, u - L1
        if 0 <= r <= H1 and 0 <= c < H1:
            return H1 * (H1 + 1) + r * H1 + c
        return -1

    # ---- build ---------------------------------------------------------------
    def _build(self):
        L, d, N, n, B = self.layout, self.d, self.N, self.n, self.B
        W, R, L1, H1 = d.W, d.R, d.L1, d.H1
        nb = self.nb
        self.org = np.zeros((nb, 4), dtype=np.int32)
        self.src = np.full((nb, W * W), -1, dtype=np.int32)
        self.gid = np.full((nb, W * W), -1, dtype=np.int64)
        self.reg = np.full((nb, W * W), -1, dtype=np.int8)
        self.nrm = np.zeros((nb, 2, NREG, W + 1, 3))
        self.lx = np.zeros((nb, H1, H1 + 1))
        self.ly = np.zeros((nb, H1 + 1, H1))
        gl: List[List[Tuple[int, int, int, int, float]]] = []
        cl: List[List[Tuple[Tuple[int, ...], Tuple[float, ...]]]] = []
        uu, vv = np.meshgrid(np.arange(W), np.arange(W))          # [v, u]
        self._need: List[List[set]] = []
        maps: Dict[Tuple[int, int], Tuple[int, np.ndarray]] = {}
        for li, tid in enumerate(self.tiles):
            face, I0, J0 = L.tile_origin(tid)
            for r_ in (REG_P, REG_W, REG_E, REG_S, REG_N):
                if (face, r_) not in maps:
                    maps[(face, r_)] = frame_map(N, face, r_)
            for yb in range(self.nby):
                for xb in range(self.nbx):
                    bid = (li * self.nby + yb) * self.nbx + xb
                    X0, Y0 = I0 + xb * B - R, J0 + yb * B - R
                    self.org[bid] = (X0, Y0, li, 0)
                    X, Y = X0 + uu, Y0 + vv
                    rg = region(X, Y, N)
                    F, I, J = neighbor_cells(N, face, X.reshape(-1), Y.reshape(-1))
                    F, I, J = F.reshape(W, W), I.reshape(W, W), J.reshape(W, W)
                    valid = rg >= 0
                    assert ((F >= 0) == valid).all()
                    g = np.where(valid, L.global_flat(F, I, J), -1)
                    self.reg[bid] = rg.reshape(-1)
                    srcv = np.full(W * W, -1, dtype=np.int64)
                    gv = g.reshape(-1)
                    m = gv >= 0
                    srcv[m] = self._source(gv[m])
                    if self._other_remote:
                        ot = L.locate(gv[m])[0] != tid
                        srcv[np.flatnonzero(m)[ot]] = -2
                    assert (srcv[m] != -1).all()
                    self.src[bid] = srcv
                    self.gid[bid] = gv
                    gslot = {int(x): k for k, x in enumerate(gv) if x >= 0}
                    self._block_geometry(bid, face, rg, F, I, J, maps)
                    gx, cx = self._block_stencils(bid, face, rg, F, I, J, g, gslot, maps, X0, Y0)
                    gl.append(gx)
                    cl.append(cx)
        G = max(1, max(len(x) for x in gl))
        C = max(1, max(len(x) for x in cl))
        self.gtab = np.zeros((nb, G, 4), dtype=np.int32)
        self.gt = np.zeros((nb, G))
        self.gcnt = np.zeros(nb, dtype=np.int32)
        self.ctab = np.full((nb, C, 6), -1, dtype=np.int32)
        self.cgeo = np.zeros((nb, C, 4))
        self.ccnt = np.zeros(nb, dtype=np.int32)
        for b in range(nb):
            self.gcnt[b] = len(gl[b])
            for k, (strip, pos, s0, s1, w) in enumerate(gl[b]):
                self.gtab[b, k] = (strip, pos, s0, s1)
                self.gt[b, k] = w
            self.ccnt[b] = len(cl[b])
            for k, (ints, flts) in enumerate(cl[b]):
                self.ctab[b, k] = ints
                self.cgeo[b, k] = flts
        # cells each stage must update (stage 0: the cells the window load must
        # provide), per block
        self.need = np.zeros((nb, d.ns + 1, W * W), dtype=bool)
        for b in range(nb):
            for s_, cells in enumerate(self._need[b]):
                self.need[b, s_, sorted(cells)] = True
        del self._need
        # strip lookup per block: [nb, 20 strips, W] -> ghost entry index or -1
        self.gidx = np.full((nb, NREG * 4, W), -1, dtype=np.int32)
        for b in range(nb):
            for k in range(self.gcnt[b]):
                s, p = self.gtab[b, k, 0], self.gtab[b, k, 1]
                self.gidx[b, s, p] = k

    def _cell_frame(self, face, rg, F, I, J, u, v, maps):
        """(panel, i, j, M) of window cell (u, v)."""
        pf, M = maps[(face, int(rg[v, u]))]
        assert pf == F[v, u]
        return int(F[v, u]), int(I[v, u]), int(J[v, u]), M

    def _block_geometry(self, bid, face, rg, F, I, J, maps):
        """Line normals and stage-1 face lengths of one block (vectorised).

        Per cell and axis: the normal and length of its face on the +axis side
        (``plus``) and on the -axis side (``minus``), both oriented +axis in the
        window, taken in the cell's own panel frame.  A face is described by its
        lower cell if that exists, else by its upper cell."""
        d = self.d
        W, L1, H1 = d.W, d.L1, d.H1
        valid = rg >= 0
        Np = np.zeros((2, W, W, 3))
        Nm = np.zeros((2, W, W, 3))
        Lp = np.zeros((2, W, W))
        Lm = np.zeros((2, W, W))
        N = self.N
        for r_ in range(NREG):
            m = rg == r_
            if not m.any():
                continue
            _, M = maps[(face, r_)]
            f, i, j = F[m], I[m], J[m]
            for axis in (0, 1):
                di, dj = M @ (np.array([1, 0]) if axis == 0 else np.array([0, 1]))
                if di == 1:
                    Np[axis][m] = self._mx[f, i + 1]
                    Nm[axis][m] = self._mx[f, i]
                    Lp[axis][m] = self._lx[f, j, i + 1]
                    Lm[axis][m] = self._lx[f, j, i]
                elif di == -1:
                    Np[axis][m] = -self._mx[f, i]
                    Nm[axis][m] = -self._mx[f, i + 1]
                    Lp[axis][m] = self._lx[f, j, i]
                    Lm[axis][m] = self._lx[f, j, i + 1]
                elif dj == 1:
                    Np[axis][m] = self._my[f, j + 1]
                    Nm[axis][m] = self._my[f, j]
                    Lp[axis][m] = self._ly[f, j + 1, i]
                    Lm[axis][m] = self._ly[f, j, i]
                else:
                    Np[axis][m] = -self._my[f, j]
                    Nm[axis][m] = -self._my[f, j + 1]
                    Lp[axis][m] = self._ly[f, j, i]
                    Lm[axis][m] = self._ly[f, j + 1, i]
        # line normals: line k between cells k-1 and k (k = 0 .. W)
        for axis in (0, 1):
            # lower cell (k-1) and upper cell (k) along the axis, for k = 0..W
            pad_r = np.full((W, 1), -1)
            if axis == 0:
                ra = np.concatenate([pad_r, rg], 1)          # [w, k]: region of (k-1, w)
                rb = np.concatenate([rg, pad_r], 1)          # region of (k, w)
                na = np.concatenate([np.zeros((W, 1, 3)), Np[0]], 1)
                nbm = np.concatenate([Nm[0], np.zeros((W, 1, 3))], 1)
            else:
                ra = np.concatenate([pad_r.T, rg], 0).T      # [w=u, k]
                rb = np.concatenate([rg, pad_r.T], 0).T
                na = np.concatenate([np.zeros((1, W, 3)), Np[1]], 0).transpose(1, 0, 2)
                nbm = np.concatenate([Nm[1], np.zeros((1, W, 3))], 0).transpose(1, 0, 2)
            rf = np.where(ra >= 0, ra, rb)
            val = np.where((ra >= 0)[..., None], na, nbm)
            ww, kk = np.nonzero(rf >= 0)
            self.nrm[bid, axis, rf[ww, kk], kk] = val[ww, kk]
        # stage-1 face lengths
        r = np.arange(H1)[:, None]
        c = np.arange(H1 + 1)[None, :]
        va, ua, ub = L1 + r, L1 + c - 1, L1 + c
        ok_a = valid[va, ua]
        self.lx[bid] = np.where(ok_a, Lp[0][va, ua], Lm[0][va, ub])
        # y-faces [line L1 + c', column L1 + r'] stored [c', r']
        ua2, vb2 = L1 + r, L1 + c                             # column, upper row
        ok_a = valid[vb2 - 1, ua2]
        ly = np.where(ok_a, Lp[1][vb2 - 1, ua2], Lm[1][vb2, ua2])   # [r' col, c' line]
        self.ly[bid] = ly.T
        self.lx[bid][~(valid[va, ua] | valid[va, ub])] = 0.0

    def _across(self, face, rg, F, I, J, u, v, side, maps):
        """Global id of the real cell across ``side`` of window cell (u, v) in
        the cell's own frame, the cell's owning tile, tile side and strip pos."""
        L = self.layout
        f, i, j, M = self._cell_frame(face, rg, F, I, J, u, v, maps)
        di, dj = M @ np.array(SIDE_VEC[side])
        F2, I2, J2 = neighbor_cells(self.N, f, np.array([i + di]), np.array([j + dj]))
        assert F2[0] >= 0
        gid = int(L.global_flat(F2[0], I2[0], J2[0]))
        tid, ti, tj = L.locate(np.array([L.global_flat(f, i, j)]))
        return gid, int(tid[0]), _side_of(di, dj), (int(tj[0]) if abs(di) == 1 else int(ti[0]))

    def _block_stencils(self, bid, face, rg, F, I, J, g, gslot, maps, X0, Y0):
        """Dependency closure of the block's step, ghost-strip entries and
        cube-corner faces.

        Working back from the block's cells (stage ns), the cells stage s - 1
        must provide are those the stage-s update of every needed cell reads:
        its partners across its four faces and the reconstruction stencils of
        both sides of each face, in each cell's own frame, where a stencil that
        crosses a panel edge reads the two cells of the interpolation pair.
        Only what is needed is tabulated, and everything needed must lie in the
        window (asserted)."""
        d = self.d
        W, N = d.W, self.N
        memo_desc: Dict[Tuple[int, int], tuple] = {}
        memo_part: Dict[Tuple[int, int], Optional[Tuple[int, int]]] = {}

        def uv(slot):
            return slot % W, slot // W

        def rg_at(u, v):
            if 0 <= u < W and 0 <= v < W:
                return int(rg[v, u])
            return int(region(X0 + u, Y0 + v, N))

        def desc(c, side):
            """Neighbour of cell c across `side` in c's own frame:
            ('slot', s) | ('interp', s0, s1, t, strip, pos); s / s0 / s1 None
            when outside the window."""
            key = (c, side)
            if key in memo_desc:
                return memo_desc[key]
            u, v = uv(c)
            du, dv = SIDE_VEC[side]
            u2, v2 = u + du, v + dv
            r_, r2 = int(rg[v, u]), rg_at(u2, v2)
            inside = 0 <= u2 < W and 0 <= v2 < W
            if r2 == r_:
                out = ("slot", v2 * W + u2 if inside else None)
            else:
                gid, tid, tside, pos = self._across(face, rg, F, I, J, u, v, side, maps)
                if inside and r2 >= 0:
                    assert gslot.get(gid) == v2 * W + u2, "index-space ghost is not the window neighbour"
                assert self._ghost_source(tid, tside, pos) == gid
                base, frac = self._pe(tid)
                b0 = int(base[tside, pos])
                s0 = gslot.get(self._ghost_source(tid, tside, b0))
                s1 = gslot.get(self._ghost_source(tid, tside, b0 + 1))
                out = ("interp", s0, s1, float(frac[tside, pos]), r_ * 4 + side, v if side < 2 else u)
            memo_desc[key] = out
            return out

        def partner(c, side):
            """(slot, side) of the cell on the other side of c's face `side`."""
            key = (c, side)
            if key in memo_part:
                return memo_part[key]
            u, v = uv(c)
            du, dv = SIDE_VEC[side]
            u2, v2 = u + du, v + dv
            r2 = rg_at(u2, v2)
            out = None
            if r2 >= 0:
                if 0 <= u2 < W and 0 <= v2 < W:
                    out = (v2 * W + u2, side ^ 1)
            else:   # beyond a cube corner: the real neighbour in c's frame
                gid, _, _, _ = self._across(face, rg, F, I, J, u, v, side, maps)
                sd = gslot.get(gid)
                if sd is not None:
                    ud, vd = uv(sd)
                    gc = int(g[v, u])
                    for s2 in range(4):
                        if rg_at(ud + SIDE_VEC[s2][0], vd + SIDE_VEC[s2][1]) >= 0:
                            continue
                        g2, _, _, _ = self._across(face, rg, F, I, J, ud, vd, s2, maps)
                        if g2 == gc:
                            out = (sd, s2)
                            break
                    assert out is not None
            memo_part[key] = out
            return out

        ghosts = {}
        corners = {}

        def stencil(x, axis, acc):
            for s_ in (2 * axis, 2 * axis + 1):
                dsc = desc(x, s_)
                if dsc[0] == "slot":
                    assert dsc[1] is not None, "stencil outside the window"
                    acc.add(dsc[1])
                else:
                    _, s0, s1, t_, strip, pos = dsc
                    assert s0 is not None and s1 is not None, "panel-edge interpolation pair outside the window"
                    acc.add(s0)
                    acc.add(s1)
                    ghosts[(strip, pos)] = (s0, s1, t_)

        ns = d.ns
        R, B = d.R, d.B
        # a cell whose cross of radius 2 lies in the window and in its own
        # region depends on exactly that cross (no panel edge within reach)
        reg_ok = np.zeros((W, W), dtype=bool)
        inner = rg[2:W - 2, 2:W - 2]
        same = inner >= 0
        for k in (-2, -1, 1, 2):
            same &= rg[2:W - 2, 2 + k:W - 2 + k] == inner
            same &= rg[2 + k:W - 2 + k, 2:W - 2] == inner
        reg_ok[2:W - 2, 2:W - 2] = same
        need = [set() for _ in range(ns + 1)]
        need[ns] = {v * W + u for v in range(R, R + B) for u in range(R, R + B)}
        for s in range(ns, 0, -1):
            lo, hi = d.stage_range(s)
            nm = np.zeros(W * W, dtype=bool)
            nm[list(need[s])] = True
            nm = nm.reshape(W, W)
            rmask = nm & reg_ok
            dil = rmask.copy()
            for k in (-2, -1, 1, 2):
                dil[:, max(k, 0):W + min(k, 0)] |= rmask[:, max(-k, 0):W + min(-k, 0)]
                dil[max(k, 0):W + min(k, 0), :] |= rmask[max(-k, 0):W + min(-k, 0), :]
            acc = set(np.flatnonzero(dil).tolist())
            for c in np.flatnonzero(nm & ~reg_ok).tolist():
                u, v = uv(c)
                assert lo <= u < hi and lo <= v < hi and rg[v, u] >= 0
                acc.add(c)
                for side in range(4):
                    p = partner(c, side)
                    assert p is not None, "face partner outside the window"
                    acc.add(p[0])
                    stencil(c, side // 2, acc)
                    stencil(p[0], p[1] // 2, acc)
                    du, dv = SIDE_VEC[side]
                    if rg_at(u + du, v + dv) < 0:
                        key = frozenset([(c, side), p])
                        if key not in corners:
                            corners[key] = ((c, side), p)
            need[s - 1] = acc
        for s in range(ns, 0, -1):
            lo, hi = d.stage_range(s)
            for c in need[s]:
                u, v = uv(c)
                assert lo <= u < hi and lo <= v < hi and rg[v, u] >= 0
        for c in need[0]:
            u, v = uv(c)
            assert rg[v, u] >= 0
        self._need.append(need)
        gout = [(strip, pos, s0, s1, t_) for (strip, pos), (s0, s1, t_) in sorted(ghosts.items())]
        cout = []
        for (c, side_c), (sd, side_d) in corners.values():
            uc, vc = uv(c)
            ud, vd = uv(sd)
            f, i, j, M = self._cell_frame(face, rg, F, I, J, uc, vc, maps)
            di, dj = M @ np.array(SIDE_VEC[side_c])
            m = self._face_normal(f, i, j, di, dj, True)          # out of c
            ln = self._face_length(f, i, j, di, dj, True)
            cout.append(((c, side_c, sd, side_d, self.fslot(uc, vc, side_c), self.fslot(ud, vd, side_d)),
                         (float(m[0]), float(m[1]), float(m[2]), ln)))
        return gout, cout


# ---------------------------------------------------------------------------
# PyTorch rendering of the fused kernel (same tables, same phases)
# ---------------------------------------------------------------------------

def _half_slope(dl, dr, lim):
    if lim == 0:
        return 0.25 * (dl + dr)
    same = dl * dr > 0
    if lim == 1:
        s = torch.sign(dl) * torch.minimum(dl.abs(), dr.abs())
    elif lim == 2:
        c = 0.5 * (dl + dr)
        s = torch.sign(c) * torch.minimum(torch.minimum(2 * dl.abs(), 2 * dr.abs()), c.abs())
    elif lim == 3:
        s = 2 * dl * dr / torch.where(same, dl + dr, torch.ones_like(dl))
    else:
        raise ValueError(f"fused step: limiter {lim} is not a PLR limiter")
    return 0.5 * torch.where(same, s, torch.zeros_like(s))


def _swe_flux(wl, wr, cl, cr, m, L, g):
    """Rusanov flux (models/swe.py::_flux), fields on dim 0, m [3, ...]."""
    hL, hR = wl[0], wr[0]
    vnL = (wl[1:] * m).sum(0)
    vnR = (wr[1:] * m).sum(0)
    sL = (cl[1:4] * m).sum(0).abs() + cl[4]
    sR = (cr[1:4] * m).sum(0).abs() + cr[4]
    c = torch.maximum(sL, sR)
    Fh = 0.5 * (hL * vnL + hR * vnR) - 0.5 * c * (hR - hL)
    Fm = 0.5 * (hL * wl[1:] * vnL + hR * wr[1:] * vnR + 0.5 * g * (hL * hL + hR * hR) * m) \
        - 0.5 * c * (hR * wr[1:] - hL * wl[1:])
    return torch.cat([Fh[None], Fm], 0) * L


class FusedTorch:
    """The fused step in PyTorch, on a SWE ``Engine`` (CPU or GPU): validates the
    host tables against the stage-by-stage oracle and documents the kernel."""

    def __init__(self, engine, plan: FusedPlan, coefs=None, remote_cells: Optional[np.ndarray] = None):
        """``remote_cells``: global ids of the receive slots (several ranks,
        ``FusedExchangePlan.need_remote[rank]``); ``step(recv)`` then takes
        their values, [slots, F]."""
        e = engine
        self.e = e
        self.p = plan
        dev, dt = e.device, e.dtype
        P = plan
        d = P.d
        W = d.W
        nb = P.nb
        self.d = d
        t = lambda a, ty=dt: torch.as_tensor(np.ascontiguousarray(a), dtype=ty, device=dev)
        self.src = t(P.src, torch.long)
        self.reg = t(P.reg.astype(np.int64), torch.long).view(nb, W, W)
        self.nrm = t(P.nrm)                                   # [nb,2,5,W+1,3]
        self.lx, self.ly = t(P.lx), t(P.ly)
        # cell records gathered through the padded layout
        tens = e.tens
        T, n, ng = e.plan.T, e.plan.n, e.plan.ng
        Pw = n + 2 * ng
        cg = torch.zeros((T, Pw, Pw, 8), dtype=dt, device=dev)
        cg[:, ng:ng + n, ng:ng + n] = tens["cgeo"]
        self.cgeo_pad = cg.view(-1, 8)
        self.S = self.cgeo_pad.shape[0]
        if remote_cells is not None and len(remote_cells):
            rec = torch.as_tensor(global_cell_records(e)[remote_cells][:, :8], dtype=dt, device=dev)
            self.cgeo_pad = torch.cat([self.cgeo_pad, rec], 0)
        self.g = float(e.physics.g)
        self.omega2 = 2.0 * float(e.physics.omega)
        self.lim = int(e.physics.limiter)
        ints = e.integ
        self.coefs = coefs or [(s.a0, s.a1, s.a2) for s in ints.stages]
        assert len(self.coefs) == d.ns
        # substitution index per (cell, side): ghost entry or -1
        gidx = torch.as_tensor(P.gidx, dtype=torch.long, device=dev)      # [nb,20,W]
        reg = self.reg
        sub = torch.full((nb, 4, W, W), -1, dtype=torch.long, device=dev)
        vv, uu = torch.meshgrid(torch.arange(W, device=dev), torch.arange(W, device=dev), indexing="ij")
        for side in range(4):
            du, dv = SIDE_VEC[side]
            u2, v2 = uu + du, vv + dv
            inside = (u2 >= 0) & (u2 < W) & (v2 >= 0) & (v2 < W)
            r2 = torch.full_like(reg, -2)
            r2[:, inside] = reg[:, v2[inside], u2[inside]]
            diff = (reg >= 0) & (r2 != reg) & (r2 != -2)
            pos = vv if side < 2 else uu
            strip = reg.clamp(min=0) * 4 + side
            k = gidx[torch.arange(nb, device=dev)[:, None, None], strip, pos[None].expand(nb, W, W)]
            sub[:, side] = torch.where(diff, k, torch.full_like(k, -1))
        self.sub = sub
        self.gt_ = torch.as_tensor(P.gtab, dtype=torch.long, device=dev)
        self.gw = t(P.gt)
        self.ctab = torch.as_tensor(P.ctab, dtype=torch.long, device=dev)
        self.cgf = t(P.cgeo)
        self.need = torch.as_tensor(P.need, device=dev).view(nb, d.ns + 1, W, W)

    def _prims(self, q):
        h = q[0]
        safe = torch.where(h != 0, h, torch.ones_like(h))
        w = torch.stack([h, q[1] / safe, q[2] / safe, q[3] / safe])
        c = torch.sqrt(self.g * torch.clamp(h, min=0.0))
        return w, c

    def step(self, recv: Optional[torch.Tensor] = None):
        e, P, d = self.e, self.p, self.d
        W, L1, H1, nb = d.W, d.L1, d.H1, P.nb
        F = 4
        Q0 = e.pool[0]
        # local cells from the padded state, remote cells (src <= -2) from recv
        rem = self.src <= -2
        srcc = torch.where(rem, self.S + (-2 - self.src), self.src).clamp(min=0)
        valid = self.need[:, 0]
        full = Q0
        if recv is not None and recv.numel():
            full = torch.cat([Q0, recv.t().to(Q0.dtype)], 1)
        q = full[:, srcc].view(F, nb, W, W) * valid
        X = q.clone()
        geo = self.cgeo_pad[srcc].view(nb, W, W, 8) * valid[..., None]
        invA = geo[..., 0]
        r = geo[..., 1:4].permute(3, 0, 1, 2)
        gb = geo[..., 4:7].permute(3, 0, 1, 2)
        bidx = torch.arange(nb, device=q.device)
        for s in range(1, d.ns + 1):
            a0, a1, a2 = self.coefs[s - 1]
            w, c = self._prims(q)
            wc = torch.cat([w, c[None]], 0)                        # [5,nb,W,W]
            # ghost strip values of this stage
            wf = w.reshape(F, nb, W * W)
            s0 = self.gt_[:, :, 2]
            s1 = self.gt_[:, :, 3]
            x0 = torch.gather(wf, 2, s0[None].expand(F, -1, -1))
            x1 = torch.gather(wf, 2, s1[None].expand(F, -1, -1))
            G = x0 + self.gw[None] * (x1 - x0)                      # [F,nb,Gmax]

            def nbr(side):
                du, dv = SIDE_VEC[side]
                sh = torch.roll(w, shifts=(-dv, -du), dims=(2, 3))
                k = self.sub[:, side]
                gv = torch.gather(G, 2, k.clamp(min=0).reshape(1, nb, -1).expand(F, -1, -1)).view(F, nb, W, W)
                return torch.where(k[None] >= 0, gv, sh)

            wm_x, wp_x, wm_y, wp_y = nbr(0), nbr(1), nbr(2), nbr(3)
            hx = _half_slope(w - wm_x, wp_x - w, self.lim)
            hy = _half_slope(w - wm_y, wp_y - w, self.lim)
            # stage-1 face set (compact): x-face (r, c) between (L1+c-1, L1+r) and (L1+c, L1+r)
            rows = slice(L1, L1 + H1)
            a_x = slice(L1 - 1, L1 + H1)
            b_x = slice(L1, L1 + H1 + 1)
            wl = (w + hx)[:, :, rows, a_x]
            wr = (w - hx)[:, :, rows, b_x]
            cl = wc[:, :, rows, a_x]
            cr = wc[:, :, rows, b_x]
            ra = self.reg[:, rows, a_x]
            rb = self.reg[:, rows, b_x]
            rf = torch.where(ra >= 0, ra, rb).clamp(min=0)
            lines = torch.arange(L1, L1 + H1 + 1, device=q.device)
            mx = self.nrm[bidx[:, None, None], 0, rf, lines[None, None, :].expand(nb, H1, H1 + 1)]   # [nb,H1,H1+1,3]
            FX = _swe_flux(wl, wr, cl, cr, mx.permute(3, 0, 1, 2), self.lx, self.g)
            FX = torch.where(((ra >= 0) & (rb >= 0))[None], FX, torch.zeros_like(FX))
            wl = (w + hy)[:, :, a_x, rows]
            wr = (w - hy)[:, :, b_x, rows]
            cl = wc[:, :, a_x, rows]
            cr = wc[:, :, b_x, rows]
            ra = self.reg[:, a_x, rows]
            rb = self.reg[:, b_x, rows]
            rf = torch.where(ra >= 0, ra, rb).clamp(min=0)
            my = self.nrm[bidx[:, None, None], 1, rf, lines[None, :, None].expand(nb, H1 + 1, H1)]
            FY = _swe_flux(wl, wr, cl, cr, my.permute(3, 0, 1, 2), self.ly, self.g)
            FY = torch.where(((ra >= 0) & (rb >= 0))[None], FY, torch.zeros_like(FY))
            # cube-corner faces
            flat = torch.cat([FX.reshape(F, nb, -1), FY.reshape(F, nb, -1)], 2)
            for b in range(nb):
                for k in range(int(P.ccnt[b])):
                    sc, side_c, sd, side_d, fc, fd = [int(x) for x in self.ctab[b, k]]
                    uc, vc, ud, vd = sc % W, sc // W, sd % W, sd // W
                    ax_c, ax_d = side_c // 2, side_d // 2
                    hc = (hx if ax_c == 0 else hy)[:, b, vc, uc]
                    hd = (hx if ax_d == 0 else hy)[:, b, vd, ud]
                    fl = w[:, b, vc, uc] + (hc if side_c % 2 else -hc)
                    fr = w[:, b, vd, ud] + (hd if side_d % 2 else -hd)
                    m = self.cgf[b, k, :3][:, None]
                    Fk = _swe_flux(fl[:, None], fr[:, None], wc[:, b, vc, uc][:, None], wc[:, b, vd, ud][:, None],
                                   m, self.cgf[b, k, 3], self.g)[:, 0]
                    if fc >= 0:
                        flat[:, b, fc] = Fk if side_c % 2 else -Fk
                    if fd >= 0:
                        flat[:, b, fd] = -Fk if side_d % 2 else Fk
            nfx = H1 * (H1 + 1)
            FX = flat[:, :, :nfx].view(F, nb, H1, H1 + 1)
            FY = flat[:, :, nfx:].view(F, nb, H1 + 1, H1)
            # cell update on the stage range
            lo, hi = d.stage_range(s)
            cs = slice(lo - L1, hi - L1)
            ce = slice(lo - L1 + 1, hi - L1 + 1)
            win = slice(lo, hi)
            iA = invA[:, win, win]
            div = (FX[:, :, cs, ce] - FX[:, :, cs, cs]) + (FY[:, :, ce, cs] - FY[:, :, cs, cs])
            dq = -div * iA
            qs = q[:, :, win, win]
            rr = r[:, :, win, win]
            hcell = qs[0]
            M = qs[1:4]
            fcor = self.omega2 * rr[2]
            cor = torch.stack([rr[1] * M[2] - rr[2] * M[1], rr[2] * M[0] - rr[0] * M[2], rr[0] * M[1] - rr[1] * M[0]])
            # curvature balance from this block's face normals and lengths
            mxw = self.nrm[:, 0]                                   # [nb,5,W+1,3]
            myw = self.nrm[:, 1]
            regw = self.reg
            # per-cell face normals: region rule "lower cell if it exists, else upper"
            def face_m(axis, plus):
                uu_ = torch.arange(lo, hi, device=q.device)
                if axis == 0:
                    k = uu_ + (1 if plus else 0)                    # line index
                    ua = (k - 1).clamp(0, W - 1)
                    ra_ = regw[:, lo:hi, :][:, :, ua]               # [nb, rows, cols]
                    rb_ = regw[:, lo:hi, :][:, :, k.clamp(max=W - 1)]
                    rf_ = torch.where(ra_ >= 0, ra_, rb_).clamp(min=0)
                    return mxw[bidx[:, None, None], rf_, k[None, None, :].expand_as(rf_)].permute(3, 0, 1, 2)
                k = uu_ + (1 if plus else 0)
                va = (k - 1).clamp(0, W - 1)
                ra_ = regw[:, :, lo:hi][:, va, :]
                rb_ = regw[:, :, lo:hi][:, k.clamp(max=W - 1), :]
                rf_ = torch.where(ra_ >= 0, ra_, rb_).clamp(min=0)
                return myw[bidx[:, None, None], rf_, k[None, :, None].expand_as(rf_)].permute(3, 0, 1, 2)

            Lw = self.lx[:, cs, cs]
            Le = self.lx[:, cs, ce]
            Ls = self.ly[:, cs, cs]
            Ln = self.ly[:, ce, cs]
            Sk = Le * face_m(0, True) - Lw * face_m(0, False) + Ln * face_m(1, True) - Ls * face_m(1, False)
            sbal = 0.5 * self.g * Sk * iA
            dq[1:] += -fcor * cor + (hcell * hcell) * sbal - self.g * hcell * gb[:, :, win, win]
            out = a2 * e.dt * dq
            if a1 != 0.0:
                out = out + a1 * qs
            if a0 != 0.0:
                out = out + a0 * X[:, :, win, win]
            dd = (out[1:4] * rr).sum(0)
            out[1:4] = out[1:4] - dd * rr
            ok = self.need[:, s, win, win][None]      # only what later stages read
            q = q.clone()
            q[:, :, win, win] = torch.where(ok, out, qs)
        # own cells -> output buffer (pool[1]), then swap
        R, B = d.R, d.B
        own = q[:, :, R:R + B, R:R + B]
        dst = self.src.view(nb, W, W)[:, R:R + B, R:R + B]
        assert (dst >= 0).all()
        Q1 = e.pool[1]
        Q1[:, dst.reshape(-1)] = own.reshape(F, -1)
        e.refresh_halos(Q1)
        e.pool[0], e.pool[1] = e.pool[1], e.pool[0]
        e.time += e.dt
        e.step_count += 1


# ---------------------------------------------------------------------------
# Device tables + descriptors of the gfx950 kernel (fused_step.hip)
# ---------------------------------------------------------------------------

FUSED_BLOCKS = (6, 8, 12, 16, 18, 20)  # block sizes the kernel is instantiated for


def rank_cus(device) -> int:
    """Compute units one rank can count on: the device's, or its share when
    STSP_SHARE_GPU=1 puts every rank of the job on one GPU (rehearsals: all
    ranks' multi-step blocks must be resident together, since a block waits
    for producers of other ranks)."""
    import os
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    if os.environ.get("STSP_SHARE_GPU") == "1":
        cus = max(1, cus // max(1, int(os.environ.get("WORLD_SIZE", "1"))))
    return cus


def fused_block(n: int, tiles: Optional[int] = None, cus: Optional[int] = None) -> Optional[int]:
    """Block size of the fused kernel for ``tiles`` tiles of n x n cells
    (None: none divides n).  With the tile count and the GPU's CU count: the
    smallest block whose blocks are all resident (one per CU: the step is one
    block's latency, which falls with the block; several steps per launch need
    every block resident), else the largest (one step per launch, fewest
    blocks).  Without them: the largest."""
    fits = [B for B in FUSED_BLOCKS if n % B == 0]
    if not fits:
        return None
    if tiles is not None and cus is not None:
        for B in fits:
            if tiles * (n // B) ** 2 <= cus:
                return B
    return fits[-1]



def fused_threads(B: int, ns: int = 3) -> int:
    """Threads per workgroup of the fused kernel (fused_step.hip FD::NT)."""
    h1 = B + 4 * (ns - 1)
    return 768 if h1 * h1 <= 768 else 1024


def stage_face_counts(B: int, ns: int = 3) -> List[int]:
    """Regular face tasks per stage after the producer wait: stage 1 only its
    outer faces (the inner ones run during the wait), then the full face sets
    of the shrinking squares (fused_step.hip: NOX, nx)."""
    h1 = B + 4 * (ns - 1)
    nil = B - 3
    out = [2 * (h1 * (h1 + 1) - nil * B)]
    for s in range(1, ns):
        nr = B + 4 * (ns - 1 - s)
        out.append(2 * nr * (nr + 1))
    return out


PASS_SLOTS = 32    # face passes per stage in the kernel's table


def pass_schedule(B: int, ncorner: np.ndarray, edge: np.ndarray, G: int, ns: int = 3,
                  weights: Optional[str] = None) -> np.ndarray:
    """[nb, ns, PASS_SLOTS] uint8: the wave that runs face pass p (faces 64 p
    .. 64 p + 63) of stage s, per block (``pass_masks`` turns it into the
    kernel's per-wave bit masks).

    The waves of a workgroup share the CU's four SIMDs as the groups
    {w, w + 4, w + 8, ...} (cyclic dispatch; tools/fused_probe.py records the
    SIMD of every wave), and a wave64 fp64 VALU instruction holds its SIMD for
    4 cycles, so a face phase lasts as long as its busiest SIMD group issues.
    Greedy balance: every pass goes to the least-loaded group, inside it to the
    least-loaded wave.  Loads in quarter passes: a regular pass 4, the cube-
    corner wave (wave 0 of a corner block) ``corner``, each ghost-entry wave
    (the waves after it in a panel-edge block) ``ghost``.  ``weights`` (or
    STSP_FUSED_SCHED) = "corner:ghost" (default "5:1": with the lane-pair
    corner faces the corner wave costs about 1.25 passes; "8:1" measured 2.5 %
    slower, profiles/r5_fused/sched_weights), or "legacy": round 4's
    placement (one pass per wave in wave order, then the second round from the
    wave after the ghost waves), kept for A/B runs."""
    import os
    weights = weights or os.environ.get("STSP_FUSED_SCHED", "5:1")
    nt = fused_threads(B, ns)
    nw = nt // 64
    counts = stage_face_counts(B, ns)
    nb = len(ncorner)
    out = np.zeros((nb, ns, PASS_SLOTS), dtype=np.uint8)
    ngw = -(-G // 64) if G > 0 else 0
    cache = {}
    for b in range(nb):
        cw = 1 if ncorner[b] > 0 else 0
        gw = ngw if edge[b] else 0
        key = (cw, gw)
        if key not in cache:
            tab = np.zeros((ns, PASS_SLOTS), dtype=np.uint8)
            for s, nt_s in enumerate(counts):
                npass = -(-nt_s // 64)
                assert npass <= PASS_SLOTS
                if weights == "legacy":
                    first = nw - cw
                    for p in range(npass):
                        tab[s, p] = p + cw if p < first else cw + gw + (p - first) % (nw - cw - gw)
                    continue
                wc, wg = (int(x) for x in weights.split(":"))
                wl = [0] * nw
                if cw:
                    wl[0] += wc
                for w in range(cw, cw + gw):
                    wl[w] += wg
                for p in range(npass):
                    gl = [sum(wl[w] for w in range(g, nw, 4)) for g in range(4)]
                    g = min(range(4), key=lambda g_: (gl[g_], g_))
                    w = min(range(g, nw, 4), key=lambda w_: (wl[w_], w_))
                    tab[s, p] = w
                    wl[w] += 4
            cache[key] = tab
        out[b] = cache[key]
    return out


def pass_masks(B: int, sched: np.ndarray, ns: int = 3, near: Optional[np.ndarray] = None) -> np.ndarray:
    """[nb, ns, 17] uint32 from ``pass_schedule``: bit p of wave w's word is
    set when w runs pass p of the stage; word 16 is the near-pass mask
    (``near_pass_masks``; fused_step.hip FArgs::sched)."""
    counts = stage_face_counts(B, ns)
    nb = sched.shape[0]
    m = np.zeros((nb, ns, 17), dtype=np.uint32)
    for s_, cnt in enumerate(counts):
        for p in range(-(-cnt // 64)):
            w = sched[:, s_, p].astype(np.int64)
            m[np.arange(nb), s_, w] |= np.uint32(1 << p)
    if near is not None:
        m[:, :, 16] = near
    return m


def stage_face_coords(B: int, ns: int = 3) -> List[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
    """Per stage, for every regular face task t of the kernel's pass loop: the
    axis (0: x-face, 1: y-face), the grid line k and the position p along it
    (window coordinates), exactly as fused_step.hip's outer_face (stage 1) and
    line-major order (stages 2, 3) map tasks."""
    d = FusedDims.make(B, ns)
    R, W, L1, H1 = d.R, d.W, d.L1, d.H1
    nil = B - 3
    ol0 = R + 2 - L1
    ol1 = (W - L1) - (R + B - 1) + 1
    nr1, nor = H1, H1 - B
    noa = (ol0 + ol1) * nr1
    nox = noa + nil * nor
    out = []
    for s_ in range(ns):
        if s_ == 0:
            nax = nox
            t = np.arange(nax)
            k = np.empty(nax, np.int64)
            p = np.empty(nax, np.int64)
            a = t < noa
            li, r = np.divmod(t[a], nr1)
            k[a] = np.where(li < ol0, L1 + li, R + B - 1 + (li - ol0))
            p[a] = L1 + r
            t2 = t[~a] - noa
            li, r = np.divmod(t2, nor)
            k[~a] = R + 2 + li
            p[~a] = np.where(r < R - L1, L1 + r, R + B + (r - (R - L1)))
        else:
            lo = R - 2 * (ns - 1 - s_)
            nr = W - 2 * lo
            nax = nr * (nr + 1)
            c, r = np.divmod(np.arange(nax), nr)
            k, p = lo + c, lo + r
        out.append((np.concatenate([np.zeros(nax, np.int64), np.ones(nax, np.int64)]),
                    np.concatenate([k, k]), np.concatenate([p, p])))
    return out


def near_pass_masks(B: int, org: np.ndarray, flags: np.ndarray, N: int, ns: int = 3) -> np.ndarray:
    """[nb, ns] uint32: bit p set when face pass p of the stage holds a face
    within one line of a panel-edge line of the block's window (the faces that
    read neighbour codes and ghost entries; fused_step.hip ``near``)."""
    nb = org.shape[0]
    out = np.zeros((nb, ns), dtype=np.uint32)
    coords = stage_face_coords(B, ns)
    far = -1000
    X0, Y0 = org[:, 0].astype(np.int64), org[:, 1].astype(np.int64)
    kx0 = np.where(flags & 2, -X0, far)
    kx1 = np.where(flags & 4, N - X0, far)
    ky0 = np.where(flags & 8, -Y0, far)
    ky1 = np.where(flags & 16, N - Y0, far)
    for s_, (ax, k, _) in enumerate(coords):
        e0 = np.where(ax[None, :] == 1, ky0[:, None], kx0[:, None])
        e1 = np.where(ax[None, :] == 1, ky1[:, None], kx1[:, None])
        kk = k[None, :]
        near = ((kk - e0 + 1 >= 0) & (kk - e0 + 1 <= 2)) | ((kk - e1 + 1 >= 0) & (kk - e1 + 1 <= 2))
        npass = -(-near.shape[1] // 64)
        for p in range(npass):
            hit = near[:, 64 * p:64 * (p + 1)].any(1)
            out[hit, s_] |= np.uint32(1 << p)
    return out


def face_normals(P: "FusedPlan", flags: np.ndarray) -> np.ndarray:
    """[nb, 3, NFL] normal of every stage-1 face slot (component-major), from
    the region line-normal tables: the region of the face's lower cell, as
    the kernel's region-table path (PFN builds read this for panel-edge
    blocks; interior blocks keep their line normals, rows left 0)."""
    d = P.d
    H1, L1 = d.H1, d.L1
    nfx = d.nfx
    nfl = 2 * nfx
    j = np.arange(nfl)
    yf = j >= nfx
    jj = np.where(yf, j - nfx, j)
    r = np.where(yf, jj // H1, jj // (H1 + 1))
    c = np.where(yf, jj - r * H1, jj - r * (H1 + 1))
    # x-face slot: row fv = L1 + r, line k = fu = L1 + c; y-face: line k = fv = L1 + r, fu = L1 + c
    fu = L1 + c
    fv = L1 + r
    k = np.where(yf, fv, fu)
    lu = fu - np.where(yf, 0, 1)          # lower cell of the face
    lv = fv - np.where(yf, 1, 0)
    ax = yf.astype(np.int64)
    out = np.zeros((P.nb, 3, nfl))
    for b in range(P.nb):
        if flags[b] == 1:
            continue
        X0, Y0 = int(P.org[b, 0]), int(P.org[b, 1])
        ra = region(X0 + lu, Y0 + lv, P.N)
        ra = np.where(ra < 0, 0, ra)
        out[b] = P.nrm[b, ax, ra, k, :].T
    return out


def fused_supported(engine, B: Optional[int] = None) -> Optional[str]:
    """None if ``engine`` can take the fused step, else the reason it cannot."""
    e = engine
    return fused_supported_config(e.physics, e.integ.name, e.layout, B)


def fused_supported_config(physics, integrator: str, layout: TileLayout, B: Optional[int] = None) -> Optional[str]:
    """``fused_supported`` from the run's configuration alone (no Engine, so no
    geometry setup: bench.py's runtime choice)."""
    from ..models.swe import ShallowWater
    if not isinstance(physics, ShallowWater):
        return "fused step: shallow water only"
    if int(physics.limiter) not in (0, 1, 2, 3):
        return "fused step: PLR limiters only (PPM runs stage by stage)"
    if integrator != "ssprk3":
        return "fused step: SSP-RK3 only"
    if layout.loopback and layout.num_ranks > 1:
        return "fused step: loopback layouts are one-rank rehearsals"
    B = B or fused_block(layout.n)
    if B is None or layout.n % B:
        return f"fused step: tile size {layout.n} is not a multiple of {' or '.join(map(str, FUSED_BLOCKS))}"
    if layout.N <= NG_PLR * 3:
        return f"fused step: C{layout.N} is too small for the ring"
    if layout.ng < NG_PLR:
        return "fused step: needs a ghost ring of 2"
    return None


class FusedKernel:
    """Device tables and the two ping-pong descriptors (pool[0] -> pool[1] and
    back) of the gfx950 fused step for a SWE ``Engine`` (HIP backend).  Every
    index the kernel dereferences is checked here, on the host.

    Several ranks: the window cells of other ranks arrive through the direct
    xGMI ring (``FusedExchangePlan``; an ``IpcRing`` allocation per rank, mapped
    by its peers): each step stores the cells peers read into their rings as
    tagged granules and reads its own remote cells from its ring, so a
    multi-GPU step is still one launch per rank and is graph-captured like a
    one-GPU step.  ``prime()`` delivers the current state (collective)."""

    def __init__(self, engine, B: Optional[int] = None, timeout_s: float = 2.0, group=None):
        from . import native
        why = fused_supported(engine, B)
        if why:
            raise RuntimeError(why)
        if B is None:
            cus = None
            if engine.device.type == "cuda":
                cus = rank_cus(engine.device)
            B = fused_block(engine.plan.n, len(engine.plan.tiles), cus)
        e = engine
        self.e = e
        self.group = group
        self.lib = native.require_native()
        self._launch_fn = self.lib.stsp_fused_launch
        world = e.layout.num_ranks
        self.world = world
        X = None
        if world > 1 or e.layout.loopback:
            X = FusedExchangePlan(e.layout, e.grid, B, ns=3)
            P = X.plans[e.rank]
        else:
            P = FusedPlan(e.layout, e.rank, e.grid, B=B, ns=3)
            P.src[~P.need[:, 0]] = -1          # load only what the step reads
        self.plan = P
        d = P.d
        W, WS, nb = d.W, d.W + 1, P.nb
        dev, dt = e.device, e.dtype
        gmax, cmax = ctypes_limits(self.lib)
        G, C = P.gtab.shape[1], P.ctab.shape[1]
        if G > gmax or C > cmax:
            raise RuntimeError(f"fused step: {G} ghost entries / {C} corner faces exceed the kernel's {gmax} / {cmax}")
        S = e.plan.S
        nring = X.ring_slots if X is not None else 0
        # ---- host-side contract checks ----------------------------------------
        assert P.src.shape == (nb, W * W) and int(P.src.max()) < S and int(P.src.min()) >= -2 - (nring - 1)
        assert (P.src[P.need[:, 0]] != -1).all()
        nfl = 2 * d.nfx
        ld = lambda s_: (s_ // W) * WS + s_ % W
        for b in range(nb):
            k = int(P.gcnt[b])
            assert (P.gtab[b, :k, 2:4] >= 0).all() and (P.gtab[b, :k, 2:4] < W * W).all()
            for j in range(int(P.ccnt[b])):
                assert -1 <= P.ctab[b, j, 4] < nfl and -1 <= P.ctab[b, j, 5] < nfl
        assert int(P.gidx.max()) < G
        code = neighbour_codes(P)
        gpair = np.zeros((nb, G, 2), dtype=np.int32)
        gpair[..., 0] = ld(P.gtab[..., 2])
        gpair[..., 1] = ld(P.gtab[..., 3])
        ct, cgw = corner_tables(P, code, gpair)
        org = P.org.copy()
        for b in range(nb):
            regs = set(int(x) for x in np.unique(P.reg[b]) if x >= 0)
            flags = sum(1 << r for r in regs)
            li, rem = divmod(b, P.nbx * P.nby)
            yb, xb = divmod(rem, P.nbx)
            face = e.layout.tile_origin(e.plan.tiles[li])[0]
            org[b, 3] = np.int32(np.uint32((xb * B) | ((yb * B) << 12) | (flags << 24) | (face << 29)).view(np.int32))
        # geometry: shared panel tables + per-block region maps (kernel_geometry);
        # grad b per cell [S (+ ring)][4] in the padded layout, only with topography
        kg = kernel_geometry(e.layout, e.grid)
        self.frames = [int(x) for x in kg["frames"]]
        t = lambda a, ty=dt: torch.as_tensor(np.ascontiguousarray(a), dtype=ty, device=dev)
        self.tens = {
            "len": t(np.concatenate([P.lx.reshape(nb, -1), P.ly.reshape(nb, -1)], 1)),
            "nrm": t(np.ascontiguousarray(np.moveaxis(P.nrm, -1, -2))),      # [nb,2,5,3,W+1]
            "tane": t(kg["tane"]), "crec": t(kg["crec"]), "lxt": t(kg["lxt"]),
            "src": t(P.src, torch.int32), "org": t(org, torch.int32),
            "code": t(code.view(np.int64), torch.int64), "gtab": t(gpair, torch.int32), "gw": t(P.gt),
            "ctab": t(ct, torch.int32), "cgf": t(cgw), "ccnt": t(P.ccnt, torch.int32),
            "push": torch.as_tensor(e.plan.push_map, dtype=torch.int32, device=dev).contiguous(),
            "cpush": torch.as_tensor(e.plan.corner_push, dtype=torch.int32, device=dev).contiguous(),
        }
        rec_g = global_cell_records(e)
        self.tens["gbt"] = None
        if np.abs(rec_g[:, 4:7]).max() > 0.0:
            T_, n, ng = e.plan.T, e.plan.n, e.plan.ng
            pw = n + 2 * ng
            gbn = np.zeros((T_, pw, pw, 4))
            L_ = e.layout
            jj, ii = np.mgrid[0:n, 0:n]
            for li, tid in enumerate(e.plan.tiles):
                f, I0, J0 = L_.tile_origin(tid)
                gbn[li, ng:ng + n, ng:ng + n, :3] = rec_g[L_.global_flat(f, I0 + ii, J0 + jj), 4:7]
            gbn = gbn.reshape(-1, 4)
            if X is not None:       # remote cells, in ring-slot order
                rg = np.zeros((len(X.need_remote[e.rank]), 4))
                rg[:, :3] = rec_g[X.need_remote[e.rank], 4:7]
                gbn = np.concatenate([gbn, rg], 0)
            self.tens["gbt"] = t(gbn)
        assert int(e.plan.push_map.max(initial=-1)) < S and int(e.plan.corner_push.max(initial=-1)) < S
        self.dcode = native.dtype_code(dt)
        self.mem = None
        # per-block step counters (xGMI tags; waits inside a multi-step launch)
        self.tens["epoch"] = torch.zeros(nb, dtype=torch.int32, device=dev)
        # tagged in-launch hand-off: [2 slots][W words][S] u64,
        # zero tags; lives with the epoch array, whose counts only grow, so a
        # tag a reader waits for was written in the same launch
        self.handoff = handoff_mode(B, multi_rank=X is not None)
        if self.handoff == "tag" and not read_relation_symmetric(P):
            if os.environ.get("STSP_FUSED_HANDOFF") == "tag":
                raise RuntimeError("tagged hand-off needs a symmetric block read relation")
            self.handoff = "epoch"
        if self.handoff == "tag" and not int(self.lib.stsp_fused_tagh()):
            if os.environ.get("STSP_FUSED_HANDOFF") == "tag":
                raise RuntimeError("STSP_FUSED_HANDOFF=tag needs a library built with STSP_FUSED_TAGH=1")
            self.handoff = "epoch"
        if self.handoff == "tag":
            # granules per cell (fused_step.hip HX<T>::W): fp64 5 (12-bit tag +
            # 52 payload bits each), fp32 4 (32-bit tag + value)
            words = 5 if e.dtype == torch.float64 else 4
            self.tens["hx"] = torch.zeros(2 * words * e.plan.S, dtype=torch.int64, device=dev)
        self.tens["err"] = torch.zeros(8, dtype=torch.int32, device=dev)   # code, block, step, what, seen
        prod = producer_table(P)
        self.tens["prod"] = torch.as_tensor(prod, dtype=torch.int32, device=dev).contiguous()
        # per-cell producer polls (epoch hand-off, one rank): every ring thread
        # waits for the producer of its own window cell, then loads it, instead
        # of wave 0 polling every producer before a barrier (profiles/r6_handoff)
        self.poll = poll_mode() if (X is None and self.handoff == "epoch" and read_relation_symmetric(P)) \
            else "block"
        if self.poll == "cell":
            self.tens["pidx"] = torch.as_tensor(cell_producer_index(P, prod), device=dev).contiguous()
        # face passes per wave, balanced over the SIMDs (pass_schedule)
        edge_b = np.array([any(int(x) > 0 for x in np.unique(P.reg[b])) for b in range(nb)])
        sched = pass_schedule(B, np.asarray(P.ccnt), edge_b, G)
        assert int(sched.max()) < fused_threads(B) // 64
        flg = (org[:, 3].view(np.uint32) >> 24) & 0x1F
        near = near_pass_masks(B, P.org, flg.astype(np.int64), e.layout.N)
        self.tens["sched"] = torch.as_tensor(pass_masks(B, sched, near=near).view(np.int32), device=dev).contiguous()
        # per-face normals of the panel-edge blocks (the kernel's PFN builds)
        self.tens["nrmf"] = t(face_normals(P, flg.astype(np.int64)))
        self.timeout_ticks = int(timeout_s * 1e8)
        if X is not None:
            self._setup_exchange(X, timeout_s)
        self.descs = [self._desc(0, 1), self._desc(1, 0)]
        self._multi = {}          # nsteps -> descriptor (pool[0] -> ... -> pool[nsteps % 2])
        self._multi_ptrs = {}     # nsteps -> (Q, out) the descriptor holds
        if X is not None:
            self.prime()

    def _setup_exchange(self, X, timeout_s: float) -> None:
        from .xgmi import IpcRing, _declare, refuse_if_forced
        refuse_if_forced()
        e = self.e
        L = _declare(self.lib)
        if int(L.stsp_xg_protocol()) != 1:
            raise RuntimeError("fused multi-rank step needs the tagged-granule protocol (STSP_XG_TAG=1)")
        self._xlib = L
        self.slots = int(L.stsp_xg_slots())
        # packed cell records (fused_step.hip HX<T>): 5 granules per fp64 cell
        self.ring = X.ring_slots * int(self.lib.stsp_fused_record_words(self.dcode))
        xpush, psrc, pcode = X.producer(e.rank)
        assert psrc.size == 0 or int(psrc.max()) < e.plan.S
        peers = sorted(set(int(c) >> XG_SLOT_BITS for c in pcode.tolist())
                       | set(int(x) for x in np.unique(np.asarray(e.layout.owner)[
                           e.layout.locate(X.need_remote[e.rank])[0]]).tolist()))
        self.mem = IpcRing(L, e.device, self.world, e.rank, peers, self.slots * self.ring * 8, self.group)
        pr = np.zeros(32, dtype=np.int64)
        for p, b in self.mem.bases.items():
            pr[p] = b
        dev = e.device
        self.tens.update({
            "peer_ring": torch.as_tensor(pr, device=dev),
            "xpush": torch.as_tensor(xpush, dtype=torch.int32, device=dev).contiguous(),
            "prime_src": torch.as_tensor(psrc, dtype=torch.int32, device=dev),
            "prime_code": torch.as_tensor(pcode, dtype=torch.int32, device=dev),
        })
        self.K = int(xpush.shape[2])

    def _desc(self, qi: int, oi: int, nsteps: int = 1):
        from . import native
        e, P, tn = self.e, self.plan, self.tens
        p = native.ptr
        d = native.FusedDesc()
        d.Q, d.out = p(e.pool[qi]), p(e.pool[oi])
        for k in ("len", "nrm", "tane", "crec", "lxt", "src", "org", "code", "gtab", "gw", "ctab", "cgf",
                  "ccnt", "push", "cpush"):
            setattr(d, k, p(tn[k]))
        d.gbt = p(tn["gbt"]) if tn["gbt"] is not None else 0
        for f in range(6):
            d.frames[f] = self.frames[f]
        d.G, d.C = P.gtab.shape[1], P.ctab.shape[1]
        d.nblocks, d.n, d.N, d.S = P.nb, e.plan.n, e.layout.N, e.plan.S
        d.mg, d.pw, d.B, d.ns = e.plan.ng, e.plan.P, P.B, P.ns
        d.limiter = int(e.physics.limiter)
        for k, st in enumerate(e.integ.stages):
            d.a0[k], d.a1[k], d.a2[k] = st.a0, st.a1, st.a2
        d.dt = e.dt
        d.g = float(e.physics.g)
        d.omega2 = 2.0 * float(e.physics.omega)
        # one rank with every tile in id order: window sources computed in the kernel
        d.local_src = 1 if (self.world == 1 and not e.layout.loopback
                            and list(e.plan.tiles) == list(range(e.layout.num_tiles))) else 0
        for f in range(6):
            d.links[f] = face_links(f)
        d.epoch = p(tn["epoch"])
        d.err = p(tn["err"])
        d.timeout_ticks = self.timeout_ticks
        d.nsteps = nsteps
        d.prod = p(tn["prod"])
        d.PM = int(tn["prod"].shape[1])
        d.sched = p(tn["sched"])
        d.nrmf = p(tn["nrmf"])
        d.hx = p(tn["hx"]) if self.handoff == "tag" else 0
        d.pidx = p(tn["pidx"]) if self.poll == "cell" else 0
        if self.mem is not None:
            d.xg = 1
            d.ring = self.ring
            d.recv = self.mem.base
            d.peer_ring = p(tn["peer_ring"])
            d.xpush = p(tn["xpush"])
            d.K = self.K
        return d

    def multi_desc(self, nsteps: int):
        """Descriptor of one launch running ``nsteps`` (even) steps from pool[0]
        (ping-pong inside the kernel; the state ends in pool[0])."""
        if nsteps < 2 or nsteps % 2:
            raise ValueError("a multi-step launch runs an even number of steps")
        d = self._multi.get(nsteps)
        if d is None:
            d = self._multi[nsteps] = self._desc(0, 1, nsteps)
            self._multi_ptrs[nsteps] = (d.Q, d.out)
        # follow the engine's current buffer order (step() swaps the pool);
        # the ctypes fields are only written when it changed (launch path)
        pp = (self.e.pool[0].data_ptr(), self.e.pool[1].data_ptr())
        if pp != self._multi_ptrs[nsteps]:
            d.Q, d.out = pp
            self._multi_ptrs[nsteps] = pp
        return d

    # ---- several ranks: delivery of the current state, error check ----------
    def prime(self) -> None:
        """Deliver the cells peers read of the current state (pool[0]) into
        their ring slot for the next step.  Collective: all ranks, quiescent."""
        if self.mem is None:
            return
        import torch.distributed as dist
        from . import native
        from .xgmi import agree
        e = self.e
        torch.cuda.synchronize(e.device)
        ep = self.tens["epoch"]
        e0 = int(ep[0].item())
        if not bool((ep == e0).all()):
            raise RuntimeError("fused xGMI epochs diverged across blocks")
        dist_on = self.mem.distributed
        if dist_on:
            dist.barrier(group=self.group)      # nobody still reads the slot we are about to fill
        tn = self.tens
        rc = self.lib.stsp_fused_prime_launch(self.dcode, native.ptr(e.pool[0]), e.plan.S,
                                              native.ptr(tn["prime_src"]), native.ptr(tn["prime_code"]),
                                              int(tn["prime_src"].numel()), native.ptr(tn["peer_ring"]), self.ring,
                                              e0, native.current_stream_handle())
        torch.cuda.synchronize(e.device)
        if not agree(rc == 0, dist_on, e.device, self.group):
            raise RuntimeError(f"fused xGMI prime failed ({rc})")
        if dist_on:
            dist.barrier(group=self.group)

    def check(self) -> None:
        w = [int(x) for x in self.tens["err"].cpu().tolist()]
        err = w[0]
        if err == 1:
            raise RuntimeError("fused step: a peer's window cells did not arrive in time (poll timeout; "
                               f"block {w[1]} at step {w[2]} waited on ring slot {w[3]}, last tag seen {w[4]})")
        if err:
            raise RuntimeError("fused step: a producer block did not finish its step in time (multi-step launch; "
                               f"block {w[1]} at step {w[2]} waited on block {w[3]}, which had finished {w[4]})")

    def close(self) -> None:
        if self.mem is not None:
            self.mem.close()
            self.mem = None

    def set_dt(self, dt: float) -> None:
        for d in list(self.descs) + list(self._multi.values()):
            d.dt = dt

    def launch(self, parity: int = 0, stream: Optional[int] = None, nsteps: int = 1) -> None:
        """One fused step from pool[parity] into pool[1 - parity] (the
        engine's pool list is not touched); nsteps > 1 (even, parity 0): that
        many steps in one launch, the state back in pool[0]."""
        d = self.descs[parity] if nsteps == 1 else self.multi_desc(nsteps)
        if stream is None:
            stream = native_stream(self.e.device)
        rc = self._launch_fn(self.dcode, d, stream)
        if rc:
            raise RuntimeError(f"fused step failed with code {rc}")

    def step(self, nsteps: int = 1) -> None:
        """Eager fused steps on the engine (state in pool[0] afterwards)."""
        e = self.e
        for _ in range(nsteps):
            self.launch(0)
            e.pool[1], e.pool[0] = e.pool[0], e.pool[1]
            self.descs = [self.descs[1], self.descs[0]]
            e.time += e.dt
            e.step_count += 1


def face_links(face: int) -> int:
    """Cube-edge links of a face for the kernel's window_src: sides W E S N,
    6 bits each: neighbour face | its edge (0 W, 1 E, 2 S, 3 N) << 3 |
    reversed << 5 (parallel/topology.py LINKS)."""
    from ..parallel.topology import LINKS
    code = 0
    for k, ed in enumerate("WESN"):
        lk = LINKS[(face, ed)]
        c = lk.nbr_face | ("WESN".index(lk.nbr_edge) << 3) | (int(lk.reversed) << 5)
        code |= c << (6 * k)
    return code


def global_cell_records(engine) -> np.ndarray:
    """[6 N N, 12] cell records of every cell of the grid, indexed by global
    flat id: 1/A, centre (3), grad b (3), the curvature sum S = sum(L m) over
    the cell's four faces with outward normals (3; the kernel's curvature
    balance is g h^2 / 2 * S / A, models/swe.py), 0, 0."""
    e = engine
    key = ("global_rec12", e.layout.N, e.physics.name, getattr(e.physics, "case", None))
    cache = getattr(e.grid, "_cache", {})
    if key in cache:
        return cache[key]
    from ..models.base import RankGeometry
    L1 = TileLayout(e.layout.N, e.layout.t, 1, ng=e.layout.ng)
    geo = RankGeometry(e.grid, L1, 0)
    rec = e.physics.setup(geo, torch.float64, "cpu")["cgeo"].numpy()          # [T, n, n, 8]
    g = e.grid
    lx, ly, mx, my = g.x_edge_lengths(), g.y_edge_lengths(), g.x_edge_normals(), g.y_edge_normals()
    Sv = (lx[:, :, 1:, None] * mx[:, None, 1:, :] - lx[:, :, :-1, None] * mx[:, None, :-1, :]
          + ly[:, 1:, :, None] * my[:, 1:, None, :] - ly[:, :-1, :, None] * my[:, :-1, None, :])   # [6,N,N,3]
    out = np.zeros((6 * L1.N * L1.N, 12))
    n = L1.n
    for li, tid in enumerate(L1.rank_tiles[0]):
        f, I0, J0 = L1.tile_origin(tid)
        jj, ii = np.mgrid[0:n, 0:n]
        gid = L1.global_flat(f, I0 + ii, J0 + jj).reshape(-1)
        out[gid, :7] = rec[li].reshape(-1, 8)[:, :7]
        out[gid, 7:10] = Sv[f, J0:J0 + n, I0:I0 + n].reshape(-1, 3)
    cache[key] = out
    return out


def neighbour_codes(P: "FusedPlan") -> np.ndarray:
    """[nb, W*W] uint64: per window cell four int16 codes (sides -x, +x, -y,
    +y): -1 = read the window neighbour (same region), >= 0 = ghost entry
    (the neighbour in the cell's own frame is the interpolation pair of that
    entry), -3 = no cell here (beyond a cube corner)."""
    W = P.d.W
    nb = P.nb
    reg = P.reg.reshape(nb, W, W).astype(np.int64)
    codes = np.full((nb, 4, W, W), -1, dtype=np.int64)
    vv, uu = np.mgrid[0:W, 0:W]
    for side in range(4):
        du, dv = SIDE_VEC[side]
        u2, v2 = uu + du, vv + dv
        inside = (u2 >= 0) & (u2 < W) & (v2 >= 0) & (v2 < W)
        pos = vv if side < 2 else uu
        for b in range(nb):
            r = reg[b]
            r2 = np.full((W, W), -2)
            r2[inside] = r[v2[inside], u2[inside]]
            diff = (r >= 0) & (r2 != r)
            strip = np.clip(r, 0, None) * 4 + side
            e = P.gidx[b, strip, pos]
            codes[b, side] = np.where(diff & (e >= 0), e, -1)
    codes[np.broadcast_to((reg < 0)[:, None], codes.shape)] = -3
    c16 = (codes & 0xFFFF).astype(np.uint64)
    out = c16[:, 0] | (c16[:, 1] << np.uint64(16)) | (c16[:, 2] << np.uint64(32)) | (c16[:, 3] << np.uint64(48))
    return out.reshape(nb, W * W)


def corner_tables(P: "FusedPlan", code: np.ndarray, gpair: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Cube-corner faces resolved for the kernel (fused_step.hip, CT_INTS /
    CG_VALS): ([nb, C, 16] int32, [nb, C, 8]).

    Per face j and side q (0: cell c, 1: cell d): ints 5q .. 5q+4 = the cell's
    LDS index, its "across" stencil neighbour as an LDS pair, its "inward"
    neighbour as a pair; 10, 11 = face slots of c and d; 12 = flags (bit 2q:
    across interpolated, 2q+1: inward interpolated, 4 + q: the face is on the
    cell's + side).  Floats: normal out of c (3), length, then the weights
    (across_c, inward_c, across_d, inward_d).  Across is the cell's neighbour
    beyond the face in its own frame (a ghost entry -> its interpolation pair
    and weight; a missing neighbour -> the cell itself), inward the one on the
    other side (the window neighbour or a ghost entry): what the kernel
    resolved from the codes at run time before round 4."""
    d = P.d
    W, WS, nb = d.W, d.W + 1, P.nb
    C = P.ctab.shape[1]
    ld = lambda s_: (s_ // W) * WS + s_ % W
    ct = np.zeros((nb, C, 16), dtype=np.int32)
    cg = np.zeros((nb, C, 8))
    for b in range(nb):
        for j in range(int(P.ccnt[b])):
            sc, side_c, sd, side_d, fc, fd = (int(x) for x in P.ctab[b, j])
            flags = 0
            for q, (cell, side) in enumerate(((sc, side_c), (sd, side_d))):
                plus = side & 1
                st = WS if side >> 1 else 1
                ic = ld(cell)
                cd = int(code[b, cell])
                nc = lambda sd_: int(np.int16(np.uint16((cd >> (16 * sd_)) & 0xFFFF)))
                eac, ein = nc(side), nc(side ^ 1)
                if eac >= 0:
                    a0, a1, ta = int(gpair[b, eac, 0]), int(gpair[b, eac, 1]), float(P.gt[b, eac])
                    flags |= 1 << (2 * q)
                else:
                    a0 = a1 = ic
                    ta = 0.0
                if ein >= 0:
                    n0, n1, tn = int(gpair[b, ein, 0]), int(gpair[b, ein, 1]), float(P.gt[b, ein])
                    flags |= 1 << (2 * q + 1)
                else:
                    n0 = n1 = ic - st if plus else ic + st
                    tn = 0.0
                flags |= plus << (4 + q)
                ct[b, j, 5 * q:5 * q + 5] = (ic, a0, a1, n0, n1)
                cg[b, j, 4 + 2 * q], cg[b, j, 5 + 2 * q] = ta, tn
            ct[b, j, 10], ct[b, j, 11], ct[b, j, 12] = fc, fd, flags
            cg[b, j, :4] = P.cgeo[b, j]
    return ct, cg


def poll_mode() -> str:
    """``STSP_FUSED_POLL`` = block (wave 0 polls every producer of the block,
    then a barrier) or cell (each ring thread polls its own cell's producer
    and loads at once); epoch hand-off on one rank only."""
    m = os.environ.get("STSP_FUSED_POLL", POLL_DEFAULT)
    if m not in ("block", "cell"):
        raise ValueError(f"STSP_FUSED_POLL must be 'block' or 'cell', got {m!r}")
    return m


POLL_DEFAULT = "block"


def cell_producer_index(P: "FusedPlan", prod: np.ndarray) -> np.ndarray:
    """[nb, W*W] int8 (window order v W + u): the index into prod[b] of the
    block that produces window cell (u, v) of block b, -1 for the block's own
    cells and cells it does not load."""
    L = P.layout
    pos = {int(t): k for k, t in enumerate(P.tiles)}
    out = np.full(P.src.shape, -1, dtype=np.int8)
    for b in range(P.nb):
        m = np.nonzero(P.src[b] >= 0)[0]
        if m.size == 0:
            continue
        tid, i, j = L.locate(P.gid[b][m])
        li = np.array([pos[int(t)] for t in tid])
        blk = (li * P.nby + j // P.B) * P.nbx + i // P.B
        where = {int(c): k for k, c in enumerate(prod[b]) if c >= 0}
        for idx, c in zip(m, blk):
            if int(c) != b:
                out[b, idx] = where[int(c)]
    return out


def read_relation_symmetric(P: "FusedPlan") -> bool:
    """True if every block whose window reads a cell of block c is itself read
    by c (in-rank producers).  The tagged hand-off waits only for the cells a
    block reads; with a symmetric relation that also keeps every producer at
    most one step ahead of its readers, which its two slots need."""
    return producer_table(P, symmetric=False)[1]


def producer_table(P: "FusedPlan", symmetric: bool = True):
    """[nb, PM] int32: the blocks of this rank whose cells each block's window
    loads (its producers for a step inside a multi-step launch), made
    symmetric so the same wait also guarantees that every reader of a block's
    previous state is done before the block overwrites it; -1 padded.
    symmetric=False: (None, whether the read relation already is symmetric)."""
    L = P.layout
    pos = {int(t): k for k, t in enumerate(P.tiles)}
    sets = [set() for _ in range(P.nb)]
    for b in range(P.nb):
        m = P.src[b] >= 0
        g = P.gid[b][m]
        if g.size == 0:
            continue
        tid, i, j = L.locate(g)
        li = np.array([pos[int(t)] for t in tid])
        blk = (li * P.nby + j // P.B) * P.nbx + i // P.B
        sets[b].update(int(x) for x in np.unique(blk) if int(x) != b)
    if not symmetric:
        return None, all(b in sets[c] for b in range(P.nb) for c in sets[b])
    for b in range(P.nb):
        for c in list(sets[b]):
            sets[c].add(b)
    PM = max(1, max(len(x) for x in sets))
    out = np.full((P.nb, PM), -1, dtype=np.int32)
    for b, x in enumerate(sets):
        out[b, :len(x)] = sorted(x)
    return out


def ctypes_limits(L) -> Tuple[int, int]:
    import ctypes
    g, c = ctypes.c_int(0), ctypes.c_int(0)
    L.stsp_fused_limits(ctypes.byref(g), ctypes.byref(c))
    return g.value, c.value


# ---------------------------------------------------------------------------
# Several ranks: remote window cells through the direct xGMI ring
# ---------------------------------------------------------------------------

def handoff_mode(B: int, multi_rank: bool = False) -> str:
    """In-launch hand-off of the in-rank cells of a multi-step fused launch
    with B x B blocks: "tag" (tagged granules, the data is the flag) or
    "epoch" (write-through state, drained per-block step counter, producer
    poll).  ``STSP_FUSED_HANDOFF`` = tag / epoch / auto (default: tag).  With
    fp64 cells packed into 5 granules of a 12-bit tag and 52 payload bits the
    tagged form is the faster one at every block size, one rank or several
    (C96 B = 16: 10.7-10.8 vs 11.8-12.1 us/step in-kernel; 8-granule tags
    lost there; profiles/r6_handoff)."""
    m = os.environ.get("STSP_FUSED_HANDOFF", "auto")
    if m not in ("tag", "epoch", "auto"):
        raise ValueError(f"STSP_FUSED_HANDOFF must be 'tag', 'epoch' or 'auto', got {m!r}")
    if m == "auto":
        return "tag"
    return m



XG_SLOT_BITS = 24


class FusedExchangePlan:
    """Which window cells of the fused step live on other ranks, and who
    stores them where (host side, numpy; tested on CPU).

    Every rank builds every rank's ``FusedPlan`` (each covers only that rank's
    blocks), so all ranks derive the same enumeration with no messages:

    * consumer p: the remote cells its blocks need (``need[0]``), ordered by
      owner rank, tile, producing block and cell, are the slots of its receive
      ring; window cells
      read them as ``src = -2 - slot``;
    * producer r: for each of its cells needed by p, the code
      ``p << 24 | slot``; the fused kernel stores the cell's new value there at
      the end of every step (tagged granules), ``xpush[block][own cell][k]``.
    """

    def __init__(self, layout: TileLayout, grid, B: int, ns: int = 3):
        L = layout
        world = L.num_ranks
        owner = np.asarray(L.owner)
        self.world = world
        # loopback (one rank, layout.loopback): the window cells of every other
        # tile travel through the rank's own ring, so one GPU runs the whole
        # xGMI protocol (tagged granules, ring slots, remote-cell geometry)
        self.loopback = bool(L.loopback) and world == 1

        def source_for(p):
            def src(g):
                tid, _, _ = L.locate(g)
                loc = L.local_flat(g)
                return np.where(owner[tid] == p, loc, -2)
            return src

        self.plans = [FusedPlan(L, p, grid, B=B, ns=ns, source=source_for(p), other_tiles_remote=self.loopback)
                      for p in range(world)]
        self.need_remote: List[np.ndarray] = []
        for p, P in enumerate(self.plans):
            m = P.need[:, 0] & (P.src == -2)
            g = np.unique(P.gid[m])
            tid, i, j = L.locate(g)
            # producer order: owner rank, tile, block row, block column, then
            # the block's cells in row order (the producing wave's lane order),
            # so the word-major ring (stage_common.h, STSP_XG_SOA) takes a
            # wave's pushes to one peer as runs of consecutive 8-byte words
            # (tools/ring_model.py)
            order = np.lexsort((i % B, j % B, i // B, j // B, tid, owner[tid]))
            self.need_remote.append(g[order])
        self.ring_slots = max(1, max(len(x) for x in self.need_remote))
        if self.ring_slots >= (1 << XG_SLOT_BITS):
            raise ValueError("receive ring too large for the push encoding")
        for p, P in enumerate(self.plans):
            slot = {int(x): k for k, x in enumerate(self.need_remote[p])}
            rem = P.src == -2
            idx = np.nonzero(rem)
            P.src[idx] = [-2 - slot[int(x)] if int(x) in slot else -1 for x in P.gid[idx]]
            # window cells nobody reads stay unloaded
            P.src[~P.need[:, 0]] = -1

    def producer(self, rank: int):
        """(xpush [nb, B*B, K] int32, prime_src [M], prime_code [M]) for ``rank``."""
        L = self.layout = self.plans[rank].layout
        P = self.plans[rank]
        B, n = P.B, P.n
        owner = np.asarray(L.owner)
        ent: Dict[int, List[int]] = {}
        psrc, pcode = [], []
        for p in range(self.world):
            if p == rank and not self.loopback:
                continue
            g = self.need_remote[p]
            tid, i, j = L.locate(g)
            mine = owner[tid] == rank
            for k in np.nonzero(mine)[0]:
                li = int(L._local_arr[tid[k]])
                x, y = int(i[k]), int(j[k])
                bid = (li * P.nby + y // B) * P.nbx + x // B
                own = (y % B) * B + x % B
                code = (p << XG_SLOT_BITS) | int(k)
                ent.setdefault(bid * B * B + own, []).append(code)
                psrc.append(int(L.local_flat(np.array([g[k]]))[0]))
                pcode.append(code)
        K = max(1, max((len(v) for v in ent.values()), default=1))
        xpush = np.full((P.nb, B * B, K), -1, dtype=np.int64)
        for key, codes in ent.items():
            b, o = divmod(key, B * B)
            xpush[b, o, :len(codes)] = codes
        return (xpush.astype(np.int32), np.asarray(psrc, dtype=np.int32), np.asarray(pcode, dtype=np.int32))
