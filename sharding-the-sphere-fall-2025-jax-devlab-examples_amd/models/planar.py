"""Single-panel shallow water on a doubly periodic f-plane (BASELINE.json
config 1: "Single-panel 32x32 shallow-water RK4 on CPU (plumbing, no GPU, no
halos)"), the "FV Cubed-Sphere Shallow Water Solver" of PY:2 reduced to one
panel.

This is the smallest end-to-end plumbing path, with the same numerics as the
cubed-sphere solver (models/swe.py):
* PLR (or PPM) faces on primitive variables;
* Rusanov fluxes;
* Coriolis;
* the explicit RK stage tables (models/integrators.py).

It runs on one flat N x N panel with periodic wrap (torch.roll), so there
are no halos and no exchange.  Conserved fields are (h, hu, hv).

Cases:
* ``rest``: a lake at rest; stays exactly steady.
* ``gaussian``: a height bump at rest; gravity waves spread symmetrically.
* ``jet``: a geostrophically balanced zonal jet, h = H + A sin(2 pi y / L),
  u = -(g / f) dh/dy.  It is steady up to truncation error.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from .base import limited_slope, ppm_faces
from .geometry import GRAVITY
from .integrators import get_integrator


def _faces_x(q: torch.Tensor, lim: int):
    """(qL, qR) at the west face of every cell (periodic in the last dim)."""
    if lim == 4:
        g, n = 3, q.shape[-1]
        qe = torch.cat([q[..., -g:], q, q[..., :g]], -1)
        aL, aR = ppm_faces(qe, g, n)          # cells -1..n
        return aR[..., :-2], aL[..., 1:-1]    # face i: right state of cell i-1, left state of cell i
    dl = q - torch.roll(q, 1, -1)
    dr = torch.roll(q, -1, -1) - q
    s = limited_slope(dl, dr, lim)
    plus = q + 0.5 * s                        # east face value of each cell
    minus = q - 0.5 * s                       # west face value
    return torch.roll(plus, 1, -1), minus


class PlanarSWE:
    name = "planar_swe"
    fields = ["h", "hu", "hv"]

    def __init__(self, N: int = 32, L: float = 1.0e6, H: float = 1000.0, case: str = "gaussian",
                 f0: float = 1.0e-4, g: float = GRAVITY, limiter: int = 2, integrator: str = "rk4",
                 dtype=torch.float64, device="cpu", cfl: float = 0.5):
        self.N, self.L, self.H, self.case = N, L, H, case
        self.f0, self.g, self.lim = f0, g, limiter
        self.dx = L / N
        self.integ = get_integrator(integrator)
        self.dtype, self.device = dtype, torch.device(device)
        x = (torch.arange(N, dtype=torch.float64) + 0.5) * self.dx
        self.Y, self.X = torch.meshgrid(x, x, indexing="ij")
        self.q = self.initial_state().to(dtype=dtype, device=self.device)
        c = math.sqrt(g * H * 1.2)
        self.dt = cfl * self.dx / (c + self.max_speed())
        self.time = 0.0
        self.step_count = 0

    # ---- state -------------------------------------------------------------
    def initial_state(self) -> torch.Tensor:
        N, L, H = self.N, self.L, self.H
        h = torch.full((N, N), H, dtype=torch.float64)
        u = torch.zeros_like(h)
        v = torch.zeros_like(h)
        if self.case == "gaussian":
            r2 = (self.X - 0.5 * L) ** 2 + (self.Y - 0.5 * L) ** 2
            h = h + 0.05 * H * torch.exp(-r2 / (0.08 * L) ** 2)
        elif self.case == "jet":
            A = 0.01 * H
            k = 2 * math.pi / L
            # cell averages of H + A sin(k y) and of the balanced u = -(g/f) A k cos(k y)
            y0, y1 = self.Y - 0.5 * self.dx, self.Y + 0.5 * self.dx
            h = H + A * (torch.cos(k * y0) - torch.cos(k * y1)) / (k * self.dx)
            u = -(self.g / self.f0) * A * (torch.sin(k * y1) - torch.sin(k * y0)) / self.dx
        elif self.case != "rest":
            raise ValueError(f"unknown planar case {self.case!r}")
        return torch.stack([h, h * u, h * v])

    def max_speed(self) -> float:
        h = self.q[0]
        return float(torch.sqrt(self.q[1] ** 2 + self.q[2] ** 2).div(h).max())

    # ---- numerics ------------------------------------------------------------
    def _flux_x(self, w: torch.Tensor, un: int) -> torch.Tensor:
        """Rusanov flux through west faces; w = (h, u, v); un = normal component (1 or 2)."""
        wL, wR = _faces_x(w, self.lim)
        g = self.g
        hL, hR = wL[0], wR[0]
        vnL, vnR = wL[un], wR[un]
        cL = torch.roll(w[un].abs() + torch.sqrt(g * w[0]), 1, -1)
        cR = w[un].abs() + torch.sqrt(g * w[0])
        a = torch.maximum(cL, cR)
        F = torch.empty_like(wL)
        F[0] = 0.5 * (hL * vnL + hR * vnR) - 0.5 * a * (hR - hL)
        for k in (1, 2):
            mL, mR = hL * wL[k], hR * wR[k]
            p = 0.5 * g * (hL * hL + hR * hR) * 0.5 if k == un else 0.0
            F[k] = 0.5 * (mL * vnL + mR * vnR) + p - 0.5 * a * (mR - mL)
        return F

    def rhs(self, q: torch.Tensor) -> torch.Tensor:
        h = q[0]
        w = torch.stack([h, q[1] / h, q[2] / h])
        Fx = self._flux_x(w, 1)                                            # west faces, x = last dim
        Gy = self._flux_x(w.transpose(-1, -2)[[0, 2, 1]], 1)              # south faces via transpose
        Gy = Gy[[0, 2, 1]].transpose(-1, -2)
        d = -((torch.roll(Fx, -1, -1) - Fx) + (torch.roll(Gy, -1, -2) - Gy)) / self.dx
        d[1] += self.f0 * q[2]
        d[2] -= self.f0 * q[1]
        return d

    def step(self, nsteps: int = 1) -> None:
        integ = self.integ
        for _ in range(nsteps):
            pool = [self.q] + [None] * (integ.nbuf - 1)
            for st in integ.stages:
                Q = pool[st.Q]
                L = self.rhs(Q)
                out = st.a2 * self.dt * L
                if st.a1:
                    out = out + st.a1 * Q
                if st.a0:
                    out = out + st.a0 * pool[st.X]
                if st.acc_out >= 0:
                    acc = st.c2 * self.dt * L
                    if st.c1:
                        acc = acc + st.c1 * pool[st.X]
                    if st.acc_in >= 0 and st.c0:
                        acc = acc + st.c0 * pool[st.acc_in]
                    pool[st.acc_out] = acc
                pool[st.out] = out
            self.q = pool[integ.rotation[0]]      # new pool[0] = old pool[rotation[0]]
            self.time += self.dt
            self.step_count += 1

    def diagnostics(self) -> Dict[str, float]:
        h, hu, hv = self.q
        A = self.dx * self.dx
        ke = 0.5 * (hu * hu + hv * hv) / h
        pe = 0.5 * self.g * h * h
        return {"mass": float(h.sum() * A), "energy": float((ke + pe).sum() * A),
                "momentum_x": float(hu.sum() * A), "momentum_y": float(hv.sum() * A)}


def run_panel(config) -> Dict[str, float]:
    """Run a single-panel config (physics.model = planar_swe)."""
    from ..utils.config import load_config
    c = load_config(config)
    dtype = {"float64": torch.float64, "fp64": torch.float64, "float32": torch.float32,
             "fp32": torch.float32}[c.grid.dtype]
    from .base import limiter_code
    m = PlanarSWE(N=c.grid.N, case=c.physics.case or "gaussian", limiter=limiter_code(c.physics.limiter),
                  integrator=c.time.integrator, dtype=dtype)
    if c.time.dt:
        m.dt = c.time.dt
    d0 = m.diagnostics()
    m.step(c.time.nsteps or 20)
    d = m.diagnostics()
    d.update({"steps": m.step_count, "time_s": m.time, "mass_rel_change": d["mass"] / d0["mass"] - 1.0})
    return d
