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

def extend(q: torch.Tensor, recv: Optional[torch.Tensor], gmap: torch.Tensor, T: int, n: int, g: int,
           ng: Optional[int] = None) -> torch.Tensor:
    """Padded state q [F, T*P*P] (P = n + 2 ng) + recv [R, F] -> extended
    window [F, T, n+2g, n+2g] with every ghost strip gathered through the ghost
    map (pull).  Corner blocks are whatever the storage holds (never read by the
    dimension-split stencils).  ``gmap`` is [T, 4, ng, n]; its first g layers
    are used."""
    F = q.shape[0]
    ng = gmap.shape[2] if ng is None else ng
    P = n + 2 * ng
    o = ng - g
    qe = q.view(F, T, P, P)[:, :, o:o + n + 2 * g, o:o + n + 2 * g].clone()
    gm = gmap[:, :, :g, :].long()
    loc = gm >= 0
    vals = q[:, gm.clamp(min=0)]                               # [F,T,4,g,n]
    if recv is not None and recv.numel() > 0:
        rv = recv[(-1 - gm).clamp(min=0)].permute(4, 0, 1, 2, 3)  # [F,T,4,g,n]
        vals = torch.where(loc.unsqueeze(0), vals, rv)
    for k in range(g):
        qe[:, :, g:g + n, g - 1 - k] = vals[:, :, 0, k, :]
        qe[:, :, g:g + n, g + n + k] = vals[:, :, 1, k, :]
        qe[:, :, g - 1 - k, g:g + n] = vals[:, :, 2, k, :]
        qe[:, :, g + n + k, g:g + n] = vals[:, :, 3, k, :]
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
    flat = (aR - qc) * (qc - aL) <= 0
    d = aR - aL
    m6 = 6.0 * (qc - 0.5 * (aL + aR))
    over_l = d * m6 > d * d
    over_r = -(d * d) > d * m6
    aL2 = torch.where(flat, qc, torch.where(over_l, 3.0 * qc - 2.0 * aR, aL))
    aR2 = torch.where(flat, qc, torch.where(~over_l & over_r, 3.0 * qc - 2.0 * aL, aR))
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
