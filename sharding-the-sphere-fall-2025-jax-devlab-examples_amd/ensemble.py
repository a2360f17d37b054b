"""Ensemble members: M independent runs of one configuration on one GPU.

SURVEY.md 2.4 lists ensembles (data parallelism over replicas) as the
optional second axis of the reference's decomposition; the reference itself
has one member (PY:19-85 builds a single 'tiles' mesh).  On MI355X a C96
stage is latency-bound: 216 blocks of one 10-wave workgroup each on 256 CUs,
plus a 1.5 us dependent-launch floor per stage (docs/ARCHITECTURE.md).
Members have no data dependence on each other, so each gets its own engine,
native runner (one hipGraph per chunk length) and HIP stream, and the
members' graphs run concurrently: one member's launch gaps and drain phases
are filled by another's blocks.  Measured at C96 fp64 (tools/ensemble_probe.py,
profiles/r2_ensemble), every member bitwise equal to the same member run alone:
one member 16.3 us/step (3.39e9 cell-updates/s); two members 22.5-23.9 us per
member step, 4.63-4.91e9 aggregate (1.38-1.45x; `python -m stsphere ensemble
configs/reference_6dev.yaml --members 2`: 4.81-4.83e9 against 3.27e9, 1.48x).  Three or more members share the
process's 4 hardware queues (GPU_MAX_HW_QUEUES) with the runners' own streams
and lose (3.2-4.1e9 for three, 2.7e9 for four), so two members per process is
the useful setting at C96.

Members differ by a relative perturbation of the initial height (field 0):
member m starts from ``q0 * (1 + amplitude * r_m)`` with ``r_m`` a fixed-seed
standard-normal field (member 0 unperturbed).
"""
from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np
import torch

from .engine import Engine
from .models.base import Physics
from .models.geometry import CubedSphereGrid
from .parallel.layout import TileLayout


class Ensemble:
    """``members`` engines of one physics / grid / layout on one device.

    backend='hip' on a GPU: each member steps through its own NativeStepper
    (graph replay) on its own stream; otherwise members step one after the
    other through ``Engine.step`` (CPU reference path)."""

    def __init__(self, physics_factory: Callable[[], Physics], layout: TileLayout, members: int,
                 amplitude: float = 1e-4, seed: int = 0, grid: Optional[CubedSphereGrid] = None,
                 dtype=torch.float64, device="cpu", backend: str = "torch", integrator: str = "ssprk3",
                 dt: Optional[float] = None, steps_per_graph: int = 100):
        if members < 1:
            raise ValueError(f"an ensemble needs at least one member, got {members}")
        if layout.num_ranks != 1:
            raise ValueError("ensemble members run whole grids on one device (layout with one rank)")
        self.grid = grid or CubedSphereGrid(layout.N)
        self.engines: List[Engine] = []
        for m in range(members):
            e = Engine(physics_factory(), layout, 0, grid=self.grid, dtype=dtype, device=device,
                       backend=backend, integrator=integrator, dt=dt)
            if dt is None:
                dt = e.dt                       # every member steps with member 0's dt
            if m > 0 and amplitude != 0.0:
                q = e.tiles_view().clone()
                g = torch.Generator().manual_seed(seed * 100003 + m)
                r = torch.randn(q[0].shape, generator=g, dtype=torch.float64).to(q.device, q.dtype)
                q[0].mul_(1.0 + amplitude * r)
                e.set_state(q)
            self.engines.append(e)
        self.dt = dt
        self.native = backend == "hip" and self.engines[0].device.type == "cuda"
        self.runners = []
        self.streams = []
        if self.native:
            from .ops.native_runtime import NativeStepper
            for e in self.engines:
                self.runners.append(NativeStepper(e, use_graph=True, steps_per_graph=steps_per_graph))
                self.streams.append(torch.cuda.Stream(e.device))

    @classmethod
    def from_config(cls, config, members: int, amplitude: float = 1e-4, seed: int = 0,
                    steps_per_graph: int = 100) -> "Ensemble":
        """Members of a run configuration (YAML path, dict or Config): the
        grid, physics, dtype, integrator and dt of ``Solver``; each member is
        a whole grid on one device (cuda:0 for ``device_type: gpu``)."""
        from .driver import make_physics
        from .models.geometry import EARTH_RADIUS
        from .utils.config import load_config
        c = load_config(config)
        gpu = c.parallelization.device_type == "gpu"
        if gpu and not torch.cuda.is_available():
            raise RuntimeError("device_type 'gpu' requested but no GPU is visible (use device_type: cpu)")
        device = torch.device("cuda:0") if gpu else torch.device("cpu")
        backend = c.runtime.backend
        if backend == "auto":
            backend = "hip" if gpu else "torch"
        dtype = {"float64": torch.float64, "fp64": torch.float64, "float32": torch.float32,
                 "fp32": torch.float32}[c.grid.dtype]
        phys0 = make_physics(c.physics)
        grid = CubedSphereGrid(c.grid.N, c.grid.radius or EARTH_RADIUS)
        layout = TileLayout(c.grid.N, c.parallelization.tiles_per_edge, 1, ng=max(c.grid.halo, phys0.halo))
        dt = c.time.dt or (phys0.max_dt(grid, c.time.cfl) if c.time.cfl else phys0.max_dt(grid))
        return cls(lambda: make_physics(c.physics), layout, members, amplitude=amplitude, seed=seed, grid=grid,
                   dtype=dtype, device=device, backend=backend, integrator=c.time.integrator, dt=dt,
                   steps_per_graph=steps_per_graph)

    @property
    def members(self) -> int:
        return len(self.engines)

    def prepare(self, nsteps: int) -> None:
        """Record (and upload) every member's graphs for ``run(nsteps)``,
        each primed on the stream it will replay on (the first replay of a
        graph on another stream pays a one-time cost again)."""
        for m, r in enumerate(self.runners):
            if m == 0:
                r.prepare(nsteps)
            else:
                with torch.cuda.stream(self.streams[m]):
                    r.prepare(nsteps)
        if self.runners:
            torch.cuda.synchronize(self.engines[0].device)

    def run(self, nsteps: int) -> None:
        """Advance every member ``nsteps`` steps.  Native: the members' graph
        replays are issued on their streams back to back and run concurrently;
        the caller's stream waits for all of them."""
        if not self.native:
            for e in self.engines:
                e.step(nsteps)
            return
        # member 0 replays on the caller's stream (a graph replayed on a side
        # stream costs ~3 us/step more at C96, docs/ARCHITECTURE.md "Graph
        # replay"), the others on their own streams, ordered after the
        # caller's earlier work
        # Launches are interleaved chunk by chunk across the members: a graph
        # exec launched again while its previous launch is still running
        # holds the host until that one is done, so issuing all of member 0's
        # chunks first would keep member 1 from starting until member 0 is
        # nearly finished (measured: no overlap at C96 with 6 chunks each).
        cur = torch.cuda.current_stream(self.engines[0].device)
        for s in self.streams[1:]:
            s.wait_stream(cur)
        per = self.runners[0].period
        chunks = [c * per for c in self.runners[0].plan(nsteps)]
        if nsteps > sum(chunks):
            chunks.append(nsteps - sum(chunks))          # partial period: eager
        for k in chunks:
            self.runners[0].run(k)
            for r, s in zip(self.runners[1:], self.streams[1:]):
                with torch.cuda.stream(s):
                    r.run(k)
        for s in self.streams[1:]:
            cur.wait_stream(s)

    def states(self) -> torch.Tensor:
        """[M, F, T, n, n] interior states of all members."""
        return torch.stack([e.tiles_view() for e in self.engines])

    def spread(self, field: int = 0) -> dict:
        """Area-weighted ensemble mean and spread (standard deviation over
        members, then RMS over the sphere) of one field."""
        x = self.states()[:, field]                              # [M, T, n, n]
        area = self.engines[0].tens["area"].reshape(x.shape[1:]).to(x.dtype)
        w = area / area.sum()
        mean = x.mean(0)
        sd = x.std(0, unbiased=False) if self.members > 1 else torch.zeros_like(mean)
        return {"mean": float((w * mean).sum()), "spread_rms": float(torch.sqrt((w * sd * sd).sum()))}

    def global_fields(self, field: int = 0) -> np.ndarray:
        """[M, 6, N, N] global field of every member (host)."""
        return np.stack([e.global_field(field) for e in self.engines])

    def close(self) -> None:
        for r in self.runners:
            r.close()
        self.runners = []
