"""Tracer advection with a prescribed wind (PDF s.13 / s.18: "Cosine Bell
Advection - Equatorial Band (PLR 2nd-Order)", "Cartesian Velocity Exchange").

    dq/dt + div(q v) = 0

PLR reconstruction + upwind edge flux  F = U * (U > 0 ? q_L : q_R),
U = (v . m) L evaluated from the Cartesian wind at each edge midpoint.
Default case: Williamson TC1 (cosine bell, alpha = 0, bell at 270 E / 0 N
starting on face 3 and moving east onto face 4, as in PDF s.18).
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch

from .base import Physics, RankGeometry, reconstruct, recon_halo
from .geometry import DAY, CubedSphereGrid
from . import initial_conditions as ic


class Advection(Physics):
    name = "advection"
    kernel_id = 0
    fields = ["q"]

    @property
    def halo(self) -> int:
        return recon_halo(self.limiter)

    def __init__(self, case: str = "cosine_bell", alpha: float = 0.0, limiter: int = 2, u0: float = None):
        self.case = case
        self.alpha = alpha
        self.limiter = limiter
        self.u0 = u0

    def _u0(self, grid):
        return self.u0 if self.u0 is not None else 2.0 * math.pi * grid.radius / (12.0 * DAY)

    def wind(self, grid, p):
        return ic.solid_body_wind(p, self._u0(grid), self.alpha, grid.radius)

    def initial_global(self, grid: CubedSphereGrid):
        p = grid.centers()
        if self.case == "cosine_bell":
            return ic.cosine_bell(p, radius=grid.radius)
        if self.case == "gaussian":
            return ic.gaussian_hill(p, center=(0.0, -1.0, 0.0), width=0.4, amp=1.0)
        if self.case == "constant":
            return np.ones(p.shape[:-1])
        raise ValueError(self.case)

    def initial_state(self, geo: RankGeometry) -> np.ndarray:
        return geo.gather_global(self.initial_global(geo.grid))[None]

    def exact(self, grid: CubedSphereGrid, t: float):
        """TC1: the bell rotated rigidly about the tilted axis; None for
        cases without a closed form."""
        if self.case != "cosine_bell":
            return None
        return ic.cosine_bell_exact(grid.centers(), t, self.alpha, radius=grid.radius, u0=self._u0(grid))

    def setup(self, geo: RankGeometry, dtype, device) -> Dict[str, torch.Tensor]:
        ux = np.sum(self.wind(geo.grid, geo.xmid) * geo.mx[:, None, :, :], axis=-1) * geo.lx
        uy = np.sum(self.wind(geo.grid, geo.ymid) * geo.my[:, :, None, :], axis=-1) * geo.ly
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=device)
        return {"area": t(geo.area), "invA": t(1.0 / geo.area), "ex": t(ux), "ey": t(uy),
                "pedge": torch.as_tensor(geo.pedge, device=device),   # [T] panel-edge side bits
                "pe_base": torch.as_tensor(geo.pe_base, device=device),   # [T,4,3,n] panel-edge ghost stencils
                "pe_t": t(geo.pe_t)}

    def kernel_params(self):
        return {"limiter": self.limiter}

    def rhs(self, qe, qi, tens, n, g):
        (qL, qR, _, _), (yL, yR, _, _) = reconstruct(qe, tens, g, n, self.limiter)
        U = tens["ex"]
        Fx = U * torch.where(U > 0, qL, qR)
        qL, qR = yL, yR
        V = tens["ey"]
        Gy = V * torch.where(V > 0, qL, qR)
        return -((Fx[..., 1:] - Fx[..., :-1]) + (Gy[..., 1:, :] - Gy[..., :-1, :])) * tens["invA"]

    def max_dt(self, grid: CubedSphereGrid, cfl: float = 0.9) -> float:
        """2-D unsplit bound dt * |v| * (1/dx + 1/dy) <= cfl."""
        return cfl * grid.min_spacing() / (2.0 * self._u0(grid))
