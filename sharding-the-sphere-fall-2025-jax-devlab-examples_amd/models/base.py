"""Physics base class, per-rank geometry, and the PyTorch reference path.

The PyTorch implementation here is the numerical oracle of the framework and
the ``device_type: cpu`` execution path (the analogue of the reference's CPU
virtual devices, PY:64-68).  The HIP kernels in ``ops/csrc`` implement the same
formulas; the GPU tests compare the two.

Finite-volume update (PDF s.4 "Finite Volume (PLR) Method"):

    dq/dt = -(1/A) [F_{i+1/2} - F_{i-1/2} + G_{j+1/2} - G_{j-1/2}] + S(q)

with piecewise-linear (PLR) reconstruction in index space along each grid
direction, a slope limiter, and physics-specific edge fluxes.  Ghost cells
come from the per-rank ghost map (``parallel/layout.py``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from ..parallel.layout import RankPlan, TileLayout
from .geometry import CubedSphereGrid, arc_angle, tangent_project

LIMITERS = {"none": 0, "central": 0, "minmod": 1, "mc": 2, "vanleer": 3, "ppm": 4}
PPM = 4          # piecewise-parabolic faces (Colella & Woodward 1984), needs halo 3


def recon_halo(lim: int) -> int:
    """Ghost layers the reconstruction reads: 2 for PLR, 3 for PPM."""
    return 3 if lim == PPM else 2


PE_LAYERS = 3    # ghost layers that carry panel-edge interpolation tables


def panel_edge_target(N: int, J: np.ndarray, k: int) -> np.ndarray:
    """Fractional along-edge index (global, in this panel's index direction)
    of the point where this panel's grid line J, extended across a panel edge
    to ghost layer k, lands on the neighbouring panel.

    Equiangular gnomonic geometry: a point at angle delta = (k + 1/2) dalpha
    beyond the edge of this panel has, on the neighbouring panel, the same
    distance delta from the edge (so the neighbour's ghost-layer cells lie on
    the right normal line), but along-edge angle
    beta' = atan(tan(beta) / tan(pi/4 + delta)), pulled toward the edge middle.
    The index-space ghost copy puts the neighbour's cell at beta instead; this
    is the kink that made PLR and PPM lose order at panel edges
    (Putman & Lin 2007, PDF s.14: ghost values by interpolation along the
    neighbouring panel's grid lines)."""
    da = 0.5 * np.pi / N
    beta = -0.25 * np.pi + (np.asarray(J, dtype=np.float64) + 0.5) * da
    delta = (k + 0.5) * da
    bp = np.arctan(np.tan(beta) / np.tan(0.25 * np.pi + delta))
    return (bp + 0.25 * np.pi) / da - 0.5


def panel_edge_tables(N: int, layout: TileLayout, tiles, layers: int):
    """Linear interpolation tables along the ghost strips that lie on panel
    edges: for tile side s (W, E, S, N), ghost layer k and strip cell j,
    the interpolated ghost is  x[b] + t (x[b+1] - x[b])  over the raw strip x
    of that layer.  The pair is chosen on the whole panel edge (global
    b in [0, N-2]), so both panels of an edge use the same stencil and the
    result does not depend on the decomposition.  Tile-local b can leave
    [0, n-2] by up to k + 1 cells (the pull toward the edge middle, k + 1/2
    cells at most); x[-1], x[-2], ... and x[n], x[n+1], ... are then the strip
    cells beyond the tile ends, the carried corner ghosts
    (parallel/layout.py::corner_sources).  At a cube corner the target is
    pulled into the strip, so no pair crosses it.
    Returns (base [T,4,layers,n] int32, t [T,4,layers,n])."""
    n, N = layout.n, layout.N
    T = len(tiles)
    base = np.zeros((T, 4, layers, n), dtype=np.int32)
    frac = np.zeros((T, 4, layers, n))
    for li, tid in enumerate(tiles):
        f, I0, J0 = layout.tile_origin(tid)
        for side in range(4):
            o = J0 if side < 2 else I0
            for k in range(layers):
                u = panel_edge_target(N, o + np.arange(n), k)
                b = np.clip(np.floor(u).astype(np.int64), 0, max(N - 2, 0))
                base[li, side, k] = b - o
                frac[li, side, k] = u - b
    return base, frac


def limiter_code(name) -> int:
    if isinstance(name, int):
        return name
    try:
        return LIMITERS[name.lower()]
    except KeyError:
        raise ValueError(f"unknown limiter {name!r}; choose from {sorted(LIMITERS)}")


class RankGeometry:
    """Float64 host geometry for the tiles of one rank (numpy)."""

    def __init__(self, grid: CubedSphereGrid, layout: TileLayout, rank: int):
        self.grid = grid
        self.layout = layout
        self.rank = rank
        self.plan: RankPlan = layout.plan(rank)
        n, N = layout.n, layout.N
        tiles = self.plan.tiles
        self.T = len(tiles)
        self.n = n
        A = grid.areas()
        C = grid.centers()
        LX = grid.x_edge_lengths()
        LY = grid.y_edge_lengths()
        MX = grid.x_edge_normals()
        MY = grid.y_edge_normals()
        XM = grid.x_edge_midpoints()
        YM = grid.y_edge_midpoints()
        self.area = np.empty((self.T, n, n))
        self.center = np.empty((self.T, n, n, 3))
        self.lx = np.empty((self.T, n, n + 1))
        self.ly = np.empty((self.T, n + 1, n))
        self.mx = np.empty((self.T, n + 1, 3))
        self.my = np.empty((self.T, n + 1, 3))
        self.xmid = np.empty((self.T, n, n + 1, 3))
        self.ymid = np.empty((self.T, n + 1, n, 3))
        self.ext1 = np.empty((self.T, n + 2, n + 2), dtype=np.int64)
        self.face = np.empty(self.T, dtype=np.int64)
        # bit s set: tile side s (W, E, S, N) lies on a cube (panel) edge
        self.pedge = np.zeros(self.T, dtype=np.int32)
        for li, tid in enumerate(tiles):
            f, I0, J0 = layout.tile_origin(tid)
            self.face[li] = f
            self.pedge[li] = (1 * (I0 == 0)) | (2 * (I0 + n == N)) | (4 * (J0 == 0)) | (8 * (J0 + n == N))
            sj, si = slice(J0, J0 + n), slice(I0, I0 + n)
            self.area[li] = A[f, sj, si]
            self.center[li] = C[f, sj, si]
            self.lx[li] = LX[f, sj, I0:I0 + n + 1]
            self.ly[li] = LY[f, J0:J0 + n + 1, si]
            self.mx[li] = MX[f, I0:I0 + n + 1]
            self.my[li] = MY[f, J0:J0 + n + 1]
            self.xmid[li] = XM[f, sj, I0:I0 + n + 1]
            self.ymid[li] = YM[f, J0:J0 + n + 1, si]
            self.ext1[li] = layout.tile_extended_index(tid, 1)
        self.pe_base, self.pe_t = panel_edge_tables(N, layout, tiles, PE_LAYERS)

    def gather_global(self, arr_global: np.ndarray) -> np.ndarray:
        """[6, N, N, ...] global array -> [T, n, n, ...] local tiles."""
        n = self.n
        out = np.empty((self.T, n, n) + arr_global.shape[3:], dtype=arr_global.dtype)
        for li, tid in enumerate(self.plan.tiles):
            f, I0, J0 = self.layout.tile_origin(tid)
            out[li] = arr_global[f, J0:J0 + n, I0:I0 + n]
        return out

    def neighbor_values(self, arr_global: np.ndarray) -> np.ndarray:
        """[T, n+2, n+2, ...] one-ring extended values from a global array."""
        flat = arr_global.reshape((-1,) + arr_global.shape[3:])
        idx = np.where(self.ext1 >= 0, self.ext1, 0)
        return flat[idx]

    def center_distances(self):
        """Great-circle distances between the true cell centres on both sides
        of every x-edge [T,n,n+1] and y-edge [T,n+1,n] (across panels too)."""
        ce = self.neighbor_values(self.grid.centers())
        n = self.n
        dx = arc_angle(ce[:, 1:n + 1, 0:n + 1], ce[:, 1:n + 1, 1:n + 2]) * self.grid.radius
        dy = arc_angle(ce[:, 0:n + 1, 1:n + 1], ce[:, 1:n + 2, 1:n + 1]) * self.grid.radius
        return dx, dy

    def fv_gradient(self, arr_global: np.ndarray) -> np.ndarray:
        """Tangent FV gradient [T,n,n,3] of a global scalar: Gauss sum of
        (edge average - cell value) m L / A (balanced: constant -> 0)."""
        ve = self.neighbor_values(arr_global)
        n = self.n
        c = ve[:, 1:n + 1, 1:n + 1]
        bx = 0.5 * (ve[:, 1:n + 1, 0:n + 1] + ve[:, 1:n + 1, 1:n + 2])   # [T,n,n+1]
        by = 0.5 * (ve[:, 0:n + 1, 1:n + 1] + ve[:, 1:n + 2, 1:n + 1])   # [T,n+1,n]
        fx = (bx[..., None] * self.lx[..., None]) * self.mx[:, None, :, :]
        fy = (by[..., None] * self.ly[..., None]) * self.my[:, :, None, :]
        s = (fx[:, :, 1:] - fx[:, :, :-1]) + (fy[:, 1:] - fy[:, :-1])
        mlx = self.lx[..., None] * self.mx[:, None, :, :]
        mly = self.ly[..., None] * self.my[:, :, None, :]
        S = (mlx[:, :, 1:] - mlx[:, :, :-1]) + (mly[:, 1:] - mly[:, :-1])
        grad = (s - c[..., None] * S) / self.area[..., None]
        return tangent_project(grad, self.center)


# ----------------------------------------------------------------------------
# Torch reference helpers
# ----------------------------------------------------------------------------

def _pull(q: torch.Tensor, recv: Optional[torch.Tensor], m: torch.Tensor) -> torch.Tensor:
    """Values [F, *m.shape] of ghost-map codes m (>= 0: padded offset in q,
    < 0: receive slot -1 - m)."""
    vals = q[:, m.clamp(min=0)]
    if recv is not None and recv.numel() > 0:
        rv = recv[(-1 - m).clamp(min=0)]
        vals = torch.where((m >= 0).unsqueeze(0), vals, rv.movedim(-1, 0))
    return vals


def extend(q: torch.Tensor, recv: Optional[torch.Tensor], gmap: torch.Tensor, T: int, n: int, g: int,
           ng: Optional[int] = None, cmap: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Padded state q [F, T*P*P] (P = n + 2 ng) + recv [R, F] -> extended
    window [F, T, n+2g, n+2g] with every ghost strip gathered through the ghost
    map (pull).  ``gmap`` is [T, 4, ng, n]; its first g layers are used.
    Corner blocks: the carried corner ghosts (panel-edge strip ends,
    ``RankPlan.corner_map`` [T, 4, ng, ng]) are gathered the same way; the rest
    is whatever the storage holds (never read by the dimension-split
    stencils)."""
    F = q.shape[0]
    ng = gmap.shape[2] if ng is None else ng
    P = n + 2 * ng
    o = ng - g
    qe = q.view(F, T, P, P)[:, :, o:o + n + 2 * g, o:o + n + 2 * g].clone()
    vals = _pull(q, recv, gmap[:, :, :g, :].long())               # [F,T,4,g,n]
    for k in range(g):
        qe[:, :, g:g + n, g - 1 - k] = vals[:, :, 0, k, :]
        qe[:, :, g:g + n, g + n + k] = vals[:, :, 1, k, :]
        qe[:, :, g - 1 - k, g:g + n] = vals[:, :, 2, k, :]
        qe[:, :, g + n + k, g:g + n] = vals[:, :, 3, k, :]
    if cmap is not None:
        cv = _pull(q, recv, cmap[:, :, :g, :g].long())             # [F,T,4,g,g] (quad, a, b)
        for quad in range(4):
            # rows a beyond the corner (S: down, N: up), columns b (W: left, E: right)
            ys = [g - 1 - a if not quad & 2 else g + n + a for a in range(g)]
            xs = [g - 1 - b if not quad & 1 else g + n + b for b in range(g)]
            for a in range(g):
                qe[:, :, ys[a], xs] = cv[:, :, quad, a, :]
    return qe


def interior(q: torch.Tensor, T: int, n: int, ng: int) -> torch.Tensor:
    """[F, T*P*P] padded -> [F, T, n, n] view of the interior cells."""
    P = n + 2 * ng
    return q.view(q.shape[0], T, P, P)[:, :, ng:ng + n, ng:ng + n]


def cells_x(qe: torch.Tensor, g: int, n: int):
    """Unreconstructed cell values left/right of the n+1 x-edges of the interior rows."""
    rows = qe[..., g:g + n, :]
    return rows[..., g - 1:g + n], rows[..., g:g + n + 1]


def cells_y(qe: torch.Tensor, g: int, n: int):
    cols = qe[..., :, g:g + n]
    return cols[..., g - 1:g + n, :], cols[..., g:g + n + 1, :]


def limited_slope(dl: torch.Tensor, dr: torch.Tensor, lim: int) -> torch.Tensor:
    if lim == 0:
        return 0.5 * (dl + dr)
    same = dl * dr > 0
    if lim == 1:
        return torch.where(same, torch.sign(dl) * torch.minimum(dl.abs(), dr.abs()), torch.zeros_like(dl))
    if lim == 2:
        c = 0.5 * (dl + dr)
        m = torch.minimum(torch.minimum(2 * dl.abs(), 2 * dr.abs()), c.abs())
        return torch.where(same, torch.sign(c) * m, torch.zeros_like(dl))
    if lim == 3:
        return torch.where(same, 2 * dl * dr / torch.where(same, dl + dr, torch.ones_like(dl)), torch.zeros_like(dl))
    raise ValueError(lim)


def ppm_faces(q: torch.Tensor, g: int, n: int, lo_edge=None, hi_edge=None):
    """PPM face values of cells -1..n of each row (q: [..., W], cell c at index
    c + g, g >= 3).  Fourth-order interface values
    a_{k-1/2} = 7/12 (q_{k-1} + q_k) - 1/12 (q_{k-2} + q_{k+1}), then the
    Colella-Woodward monotonicity limiter.  Returns (aL, aR) each [..., n+2].

    Panel edges: grid lines bend where two cube faces meet, so a 4-cell
    stencil across a panel edge samples a kinked line and the interface value
    drops to first order there (measured on TC2).  Cells whose stencil crosses
    a panel edge (lo_edge / hi_edge: bool, broadcastable to q[..., :1], true
    where the row's low / high end is a panel edge) therefore use the MC-limited
    PLR faces instead, the usual second-order edge treatment."""
    def cell(c0, c1):          # cells c0..c1-1
        return q[..., c0 + g:c1 + g]
    # interfaces k - 1/2 for k = -1 .. n + 1 (between cells k - 1 and k)
    a = (7.0 / 12.0) * (cell(-2, n + 1) + cell(-1, n + 2)) - (1.0 / 12.0) * (cell(-3, n) + cell(0, n + 3))
    aL, aR = a[..., :-1], a[..., 1:]
    qc = cell(-1, n + 1)
    aL2, aR2 = ppm_limit(qc, aL, aR)
    if lo_edge is not None or hi_edge is not None:
        s = 0.5 * limited_slope(qc - cell(-2, n), cell(0, n + 2) - qc, 2)
        x = torch.arange(-1, n + 1, device=q.device)
        near = torch.zeros(q.shape[:-1] + (n + 2,), dtype=torch.bool, device=q.device)
        if lo_edge is not None:
            near = near | (lo_edge & (x <= 1))
        if hi_edge is not None:
            near = near | (hi_edge & (x >= n - 2))
        aL2 = torch.where(near, qc - s, aL2)
        aR2 = torch.where(near, qc + s, aR2)
    return aL2, aR2


def plr_x(qe: torch.Tensor, g: int, n: int, lim: int, pedge: Optional[torch.Tensor] = None):
    """Left/right PLR (or PPM, lim = 4) states at the n+1 x-edges of the
    interior rows: returns (qL, qR) each [..., n, n+1].  qe: [..., T, W, W];
    pedge: [T] panel-edge side bits (RankGeometry.pedge), used by PPM."""
    rows = qe[..., g:g + n, :]
    if lim == PPM:
        if g < 3:
            raise ValueError("PPM reconstruction needs a halo of 3")
        lo = hi = None
        if pedge is not None:
            lo = ((pedge & 1) != 0)[:, None, None]
            hi = ((pedge & 2) != 0)[:, None, None]
        aL, aR = ppm_faces(rows, g, n, lo, hi)    # cells -1..n
        return aR[..., :-1], aL[..., 1:]
    d = rows[..., 1:] - rows[..., :-1]
    s = limited_slope(d[..., g - 2:g + n], d[..., g - 1:g + n + 1], lim)
    c = rows[..., g - 1:g + n + 1]
    return (c + 0.5 * s)[..., :-1], (c - 0.5 * s)[..., 1:]


def plr_y(qe: torch.Tensor, g: int, n: int, lim: int, pedge: Optional[torch.Tensor] = None):
    """(qL, qR) each [..., n+1, n] at the y-edges of the interior columns."""
    pe = None if pedge is None else (pedge >> 2)      # S, N bits -> low, high
    qL, qR = plr_x(qe.transpose(-1, -2), g, n, lim, pe)
    return qL.transpose(-1, -2), qR.transpose(-1, -2)


def _strip(w: torch.Tensor, side: int, k: int, g: int, n: int) -> torch.Tensor:
    """Ghost layer k of tile side (0 W, 1 E, 2 S, 3 N) of a window [..., T, W, W]
    as [..., T, n] (along-strip index in the panel's index direction)."""
    if side == 0:
        return w[..., g:g + n, g - 1 - k]
    if side == 1:
        return w[..., g:g + n, g + n + k]
    if side == 2:
        return w[..., g - 1 - k, g:g + n]
    return w[..., g + n + k, g:g + n]


def _strip_ext(w: torch.Tensor, side: int, k: int, g: int, n: int) -> torch.Tensor:
    """Ghost layer k of a side over the whole window, [..., T, n + 2g]: along
    positions -g .. n+g-1 (the ends are corner ghosts, carried on panel
    edges)."""
    if side == 0:
        return w[..., :, g - 1 - k]
    if side == 1:
        return w[..., :, g + n + k]
    if side == 2:
        return w[..., g - 1 - k, :]
    return w[..., g + n + k, :]


def _own_ext(w: torch.Tensor, side: int, k: int, g: int, n: int) -> torch.Tensor:
    """The cells at depth k from side (k = 0: the edge cells) over the whole
    window, along positions -g .. n+g-1 (the ends are the neighbouring tiles'
    ghosts), [..., T, n + 2g]."""
    if side == 0:
        return w[..., :, g + k]
    if side == 1:
        return w[..., :, g + n - 1 - k]
    if side == 2:
        return w[..., g + k, :]
    return w[..., g + n - 1 - k, :]


def _interp(x: torch.Tensor, b: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """x [..., T, m]; b, t [T, n]: x[b] + t (x[b+1] - x[b]) along the last axis."""
    idx = b.long().expand(x.shape[:-1] + b.shape[-1:])
    x0 = x.gather(-1, idx)
    x1 = x.gather(-1, idx + 1)
    return x0 + t * (x1 - x0)


def ppm_limit(qc, aL, aR):
    """Colella-Woodward monotonicity limiter of a cell's interface values."""
    flat = (aR - qc) * (qc - aL) <= 0
    d = aR - aL
    m6 = 6.0 * (qc - 0.5 * (aL + aR))
    over_l = d * m6 > d * d
    over_r = -(d * d) > d * m6
    aL2 = torch.where(flat, qc, torch.where(over_l, 3.0 * qc - 2.0 * aR, aL))
    aR2 = torch.where(flat, qc, torch.where(~over_l & over_r, 3.0 * qc - 2.0 * aL, aR))
    return aL2, aR2


def _inner_face(line, lim: int):
    """Face value, on the side of index g - 1, of the cell at index g of a
    1-D line [..., 2g] (cells g-1, g-2, ... are on the other panel)."""
    g = line.shape[-1] // 2
    c, l, r = line[..., g], line[..., g - 1], line[..., g + 1]
    if lim == PPM:
        l2, r2 = line[..., g - 2], line[..., g + 2]
        aL = (7.0 / 12.0) * (l + c) - (1.0 / 12.0) * (l2 + r)
        aR = (7.0 / 12.0) * (c + r) - (1.0 / 12.0) * (l + r2)
        return ppm_limit(c, aL, aR)[0]
    return c - 0.5 * limited_slope(c - l, r - c, lim)


def reconstruct(w: torch.Tensor, tens: Dict[str, torch.Tensor], g: int, n: int, lim: int):
    """Edge states of the interior x- and y-edges with the panel-edge
    treatment.  w: window [F, T, W, W] with raw (index-space copy) ghosts.

    * Ghost strips on panel edges are replaced by linear interpolation along
      the strip to where this panel's grid lines really cross into the
      neighbour (``panel_edge_tables``); every face of this tile's cells is then
      reconstructed on straight grid lines (PLR, or PPM without any fallback).
    * The neighbour's state at a panel edge is reconstructed in the neighbour's
      own frame: on the line [its ghosts = our cells interpolated at its grid
      lines | its real cells].  Both panels evaluate the same pair of states at
      their common edge, so the flux is single-valued (conservative).
    * The cell values returned for wave-speed estimates are real cells on both
      sides of every edge.

    Returns (xL, xR, cxL, cxR) at the x-edges [F,T,n,n+1] and (yL, yR, cyL, cyR)
    at the y-edges [F,T,n+1,n]."""
    pe = tens.get("pedge")
    if pe is None or "pe_base" not in tens:
        xL, xR = plr_x(w, g, n, lim, pe)
        yL, yR = plr_y(w, g, n, lim, pe)
        return (xL, xR) + cells_x(w, g, n), (yL, yR) + cells_y(w, g, n)
    base, frac = tens["pe_base"], tens["pe_t"]
    wi = w.clone()
    faces = {}
    for side in range(4):
        m = ((pe >> side) & 1) != 0
        if not bool(m.any()):
            continue
        mk = m[:, None]
        gp, raw = [], []
        for k in range(g):
            # pair (b, b + 1), tile-local b >= -g: index b + g of the whole
            # window line
            b, t = base[:, side, k] + g, frac[:, side, k]
            x = _strip(w, side, k, g, n)
            raw.append(x)
            _strip(wi, side, k, g, n).copy_(torch.where(mk, _interp(_strip_ext(w, side, k, g, n), b, t), x))
            gp.append(_interp(_own_ext(w, side, k, g, n), b, t))
        line = torch.stack(gp[::-1] + raw, -1)              # [F,T,n,2g]
        faces[side] = (m, _inner_face(line, lim), raw[0])
    xL, xR = plr_x(wi, g, n, lim)
    yL, yR = plr_y(wi, g, n, lim)
    cxL, cxR = cells_x(w, g, n)
    cyL, cyR = cells_y(w, g, n)
    for side, (m, fv, r0) in faces.items():
        mk = m[:, None]
        if side == 0:
            xL[..., 0] = torch.where(mk, fv, xL[..., 0])
        elif side == 1:
            xR[..., n] = torch.where(mk, fv, xR[..., n])
        elif side == 2:
            yL[..., 0, :] = torch.where(mk, fv, yL[..., 0, :])
        else:
            yR[..., n, :] = torch.where(mk, fv, yR[..., n, :])
    return (xL, xR, cxL, cxR), (yL, yR, cyL, cyR)


class Physics:
    """Base class.  Subclasses define fields, halo need and the reference RHS."""

    name = "base"
    kernel_id = -1
    fields: List[str] = []
    halo = 2

    @property
    def F(self) -> int:
        return len(self.fields)

    def setup(self, geo: RankGeometry, dtype: torch.dtype, device) -> Dict[str, torch.Tensor]:
        raise NotImplementedError

    def initial_state(self, geo: RankGeometry) -> np.ndarray:
        """[F, T, n, n] float64."""
        raise NotImplementedError

    def rhs(self, qe: torch.Tensor, qi: torch.Tensor, tens: Dict[str, torch.Tensor], n: int, g: int) -> torch.Tensor:
        """qe: extended window [F,T,n+2g,n+2g]; qi: interior [F,T,n,n].
        Returns dq/dt [F,T,n,n]."""
        raise NotImplementedError

    def finalize(self, out: torch.Tensor, tens: Dict[str, torch.Tensor]) -> torch.Tensor:
        """Post-stage fix-up on an interior tensor [F,T,n,n] (in place)."""
        return out

    def kernel_params(self) -> Dict[str, float]:
        return {}

    def max_dt(self, grid: CubedSphereGrid, cfl: float = 0.8) -> float:
        raise NotImplementedError

    def diagnostics(self, qi: torch.Tensor, tens: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Per-rank partial sums over the interior qi [F,T,n,n] (to be all-reduced)."""
        return {"mass": (qi[0] * tens["area"]).sum()}
