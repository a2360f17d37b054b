"""Thermal diffusion on the sphere (PDF s.12 / s.17: "Lima Flag Temperature
Diffusion", checkerboard heat source on the top panel, day 0.4 -> day 26.7).

    dT/dt = div(kappa grad T)

Two-point flux  F = -kappa (T_R - T_L) L / d  across every edge, with d the
great-circle distance between the true cell centres on both sides (across
panel edges too), so the scheme is exactly conservative and symmetric.
Needs a one-cell halo (the reference's (N+2)^2 layout, PY:141).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from .base import Physics, RankGeometry
from .geometry import CubedSphereGrid
from . import initial_conditions as ic


class Diffusion(Physics):
    name = "diffusion"
    kernel_id = 1
    fields = ["T"]
    halo = 1

    def __init__(self, kappa: float = 2.0e6, case: str = "lima_flag", squares: int = 8):
        self.kappa = kappa
        self.case = case
        self.squares = squares

    def initial_global(self, grid: CubedSphereGrid):
        if self.case == "lima_flag":
            return ic.lima_flag(grid.N, self.squares)
        if self.case == "gaussian":
            return ic.gaussian_hill(grid.centers())
        raise ValueError(self.case)

    def initial_state(self, geo: RankGeometry) -> np.ndarray:
        return geo.gather_global(self.initial_global(geo.grid))[None]

    def setup(self, geo: RankGeometry, dtype, device) -> Dict[str, torch.Tensor]:
        dx, dy = geo.center_distances()
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=device)
        self._coef = (self.kappa * geo.lx / dx, self.kappa * geo.ly / dy, geo.area)
        return {"area": t(geo.area), "invA": t(1.0 / geo.area),
                "ex": t(self.kappa * geo.lx / dx), "ey": t(self.kappa * geo.ly / dy)}

    def rhs(self, qe, qi, tens, n, g):
        c = qe[..., g:g + n, g - 1:g + n + 1]
        Fx = -tens["ex"] * (c[..., 1:] - c[..., :-1])
        c = qe[..., g - 1:g + n + 1, g:g + n]
        Gy = -tens["ey"] * (c[..., 1:, :] - c[..., :-1, :])
        return -((Fx[..., 1:] - Fx[..., :-1]) + (Gy[..., 1:, :] - Gy[..., :-1, :])) * tens["invA"]

    def max_dt(self, grid: CubedSphereGrid, cfl: float = 0.8) -> float:
        # forward-Euler bound dt * sum_e(kappa L_e / d_e) / A <= 1  ~  dx^2 / (4 kappa)
        return cfl * grid.min_spacing() ** 2 / (4.0 * self.kappa)
