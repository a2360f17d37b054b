"""Shallow-water equations on the cubed sphere (PY:2 "FV Cubed-Sphere Shallow
Water Solver").

Formulation (chosen here; the reference does not show one):

* state per cell: depth h and **Cartesian momentum** M = h v (3 components),
  panel-invariant, so halos need no basis rotation (PDF s.18, "Cartesian
  Velocity Exchange");
* flux form  d(h, M)/dt + div(h v, M v + g h^2/2 I) = S,  FV with PLR on the
  primitive variables (h, v) and a Rusanov (local Lax-Friedrichs) edge flux
  along the exact great-circle edge normals; the Rusanov speed is
  max(|v.m| + sqrt(g h)) over the two adjacent cell averages;
* sources: Coriolis  -f r x M  (f = 2 Omega z/R), topography  -g h grad b, and
  the curvature balance  +g h_c^2 / 2 * (sum m L) / A, which makes a constant
  depth exactly force-free on the curved cell;
* after each stage M is projected onto the tangent plane at the cell centre
  (removes the radial "constraint force" of motion on the sphere).
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch

from .base import Physics, RankGeometry, reconstruct, recon_halo
from .geometry import GRAVITY, OMEGA, CubedSphereGrid
from . import initial_conditions as ic


class ShallowWater(Physics):
    name = "swe"
    kernel_id = 2
    fields = ["h", "mx", "my", "mz"]

    @property
    def halo(self) -> int:
        return recon_halo(self.limiter)

    def __init__(self, case: str = "tc5", limiter: int = 2, g: float = GRAVITY, omega: float = OMEGA,
                 alpha: float = 0.0):
        self.case = case
        self.limiter = limiter
        self.g = g
        self.omega = omega
        self.alpha = alpha
        self._b_global = None

    # ---- initial conditions --------------------------------------------
    def global_fields(self, grid: CubedSphereGrid):
        p = grid.centers()
        if self.case == "tc2":
            h, wind, b = ic.williamson_tc2(p, alpha=self.alpha, radius=grid.radius, omega=self.omega, g=self.g)
        elif self.case == "tc5":
            h, wind, b = ic.williamson_tc5(p, radius=grid.radius, omega=self.omega, g=self.g)
        elif self.case == "tc6":
            h, wind, b = ic.williamson_tc6(p, radius=grid.radius, omega=self.omega, g=self.g)
        elif self.case == "rest":
            h = np.full(p.shape[:-1], 1000.0)
            wind = np.zeros(p.shape)
            b = np.zeros(p.shape[:-1])
        else:
            raise ValueError(f"unknown SWE case {self.case!r}")
        return h, wind, b

    def exact(self, grid: CubedSphereGrid, t: float):
        """True depth h(t) where the case has one: TC2 (steady geostrophic
        flow) and the lake at rest keep their initial depth; else None."""
        if self.case in ("tc2", "rest"):
            return self.global_fields(grid)[0]
        return None

    def initial_state(self, geo: RankGeometry) -> np.ndarray:
        h, wind, b = self.global_fields(geo.grid)
        hl = geo.gather_global(h)
        wl = geo.gather_global(wind)
        q = np.empty((4,) + hl.shape)
        q[0] = hl
        q[1:] = np.moveaxis(hl[..., None] * wl, -1, 0)
        return q

    # ---- geometry ---------------------------------------------------------
    def setup(self, geo: RankGeometry, dtype, device) -> Dict[str, torch.Tensor]:
        _, _, b = self.global_fields(geo.grid)
        gb = geo.fv_gradient(b)
        # curvature balance  g/2 * sum_e(+-L_e m_e) / A  per cell (metric term)
        mlx = geo.lx[..., None] * geo.mx[:, None, :, :]
        mly = geo.ly[..., None] * geo.my[:, :, None, :]
        S = (mlx[:, :, 1:] - mlx[:, :, :-1]) + (mly[:, 1:] - mly[:, :-1])
        sbal = 0.5 * self.g * S / geo.area[..., None]
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=device)
        return {
            "area": t(geo.area),
            "invA": t(1.0 / geo.area),
            "ex": t(geo.lx),
            "ey": t(geo.ly),
            "mx": t(np.moveaxis(geo.mx, -1, 1)),           # [T,3,n+1]
            "my": t(np.moveaxis(geo.my, -1, 1)),
            "ctr": t(np.moveaxis(geo.center, -1, 0)),      # [3,T,n,n]
            "gradb": t(np.moveaxis(gb, -1, 0)),            # [3,T,n,n]
            "sbal": t(np.moveaxis(sbal, -1, 0)),           # [3,T,n,n]
            # HIP kernel: one 16-byte-aligned record per cell (1/A, centre, grad b, 0)
            "cgeo": t(np.concatenate([(1.0 / geo.area)[..., None], geo.center, gb,
                                      np.zeros(geo.area.shape + (1,))], axis=-1)),   # [T,n,n,8]
            "b": t(geo.gather_global(b)),
            "pedge": torch.as_tensor(geo.pedge, device=device),   # [T] panel-edge side bits
            "pe_base": torch.as_tensor(geo.pe_base, device=device),   # [T,4,3,n] panel-edge ghost stencils
            "pe_t": t(geo.pe_t),
        }

    def kernel_params(self):
        return {"g": self.g, "omega2": 2.0 * self.omega, "limiter": self.limiter}

    # ---- reference RHS ------------------------------------------------------
    def _flux(self, wL, wR, cL, cR, m, L):
        g = self.g
        hL, hR = wL[0], wR[0]
        vL, vR = wL[1:], wR[1:]
        vnL = (vL * m).sum(0)
        vnR = (vR * m).sum(0)
        sL = ((cL[1:] * m).sum(0)).abs() + torch.sqrt(g * cL[0])
        sR = ((cR[1:] * m).sum(0)).abs() + torch.sqrt(g * cR[0])
        c = torch.maximum(sL, sR)
        Fh = 0.5 * (hL * vnL + hR * vnR) - 0.5 * c * (hR - hL)
        Fm = 0.5 * (hL * vL * vnL + hR * vR * vnR + 0.5 * g * (hL * hL + hR * hR) * m) - 0.5 * c * (hR * vR - hL * vL)
        return torch.cat([Fh[None], Fm], 0) * L

    def rhs(self, qe, qi, tens, n, g):
        h = qe[0]
        safe = torch.where(h != 0, h, torch.ones_like(h))
        w = torch.stack([h, qe[1] / safe, qe[2] / safe, qe[3] / safe])
        (wL, wR, cL, cR), (yL, yR, dL, dR) = reconstruct(w, tens, g, n, self.limiter)   # x: [4,T,n,n+1]
        mx = tens["mx"].permute(1, 0, 2)[:, :, None, :]              # [3,T,1,n+1]
        Fx = self._flux(wL, wR, cL, cR, mx, tens["ex"])
        wL, wR, cL, cR = yL, yR, dL, dR                             # y: [4,T,n+1,n]
        my = tens["my"].permute(1, 0, 2)[:, :, :, None]              # [3,T,n+1,1]
        Gy = self._flux(wL, wR, cL, cR, my, tens["ey"])
        invA = tens["invA"]
        dq = -((Fx[..., 1:] - Fx[..., :-1]) + (Gy[..., 1:, :] - Gy[..., :-1, :])) * invA
        hc = qi[0]
        M = qi[1:4]
        r = tens["ctr"]
        f = self.omega * 2.0 * r[2]
        cor = torch.stack([r[1] * M[2] - r[2] * M[1], r[2] * M[0] - r[0] * M[2], r[0] * M[1] - r[1] * M[0]])
        dq[1:] += -f * cor + (hc * hc) * tens["sbal"] - self.g * hc * tens["gradb"]
        return dq

    def finalize(self, out, tens):
        r = tens["ctr"]
        M = out[1:4]
        d = (M * r).sum(0)
        out[1:4] = M - d * r
        return out

    def max_dt(self, grid: CubedSphereGrid, cfl: float = 0.9) -> float:
        """2-D unsplit bound: dt * speed * (1/dx + 1/dy) <= cfl."""
        h, wind, b = self.global_fields(grid)
        speed = np.linalg.norm(wind, axis=-1) + np.sqrt(self.g * np.maximum(h, 0))
        return cfl * grid.min_spacing() / (2.0 * float(speed.max()))

    def diagnostics(self, qi, tens):
        A = tens["area"]
        h = qi[0]
        M = qi[1:4]
        b = tens["b"]
        ke = 0.5 * (M * M).sum(0) / h
        pe = 0.5 * self.g * h * h + self.g * h * b
        return {"mass": (h * A).sum(), "energy": ((ke + pe) * A).sum()}
