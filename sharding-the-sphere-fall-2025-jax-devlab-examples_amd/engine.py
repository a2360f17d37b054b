"""Per-rank execution engine: state buffers, integrator stages, halo phases.

One ``Engine`` per rank (one process per GPU, or one virtual rank in-process).
A time step is the integrator's stage list; each stage is

    transport.start(Q)      pack boundary cells, post P2P messages
    compute(interior)       HIP: blocks that read no remote ghost
    recv = transport.finish()
    compute(boundary)       the remaining blocks (gather from recv)

With ``backend='torch'`` compute is the PyTorch reference (CPU or GPU); with
``backend='hip'`` it is the fused gfx950 stage kernel (``ops/csrc``), and the
``NativeRuntime`` can take over the whole step loop (C++ + hipGraph + RCCL).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .models.base import Physics, RankGeometry, extend, interior
from .models.geometry import CubedSphereGrid
from .models.integrators import Integrator, Stage, get_integrator
from .parallel.comm import NullTransport, Transport
from .parallel.layout import TileLayout


class TorchCompute:
    """Reference stage computation in PyTorch."""

    def __init__(self, engine: "Engine"):
        self.e = engine

    def stage(self, st: Stage, dt: float, recv: Optional[torch.Tensor], part: str = "all") -> None:
        if part == "interior":
            return  # torch path computes everything in the "boundary" call
        e = self.e
        phys = e.physics
        Q = e.pool[st.Q]
        g = phys.halo
        qe = extend(Q, recv, e.gmap, e.plan.T, e.plan.n, g, cmap=e.cmap)
        Qi = e.interior(Q)
        Xi = e.interior(e.pool[st.X])
        dq = phys.rhs(qe, Qi, e.tens, e.plan.n, g)
        if st.acc_out >= 0:
            acc = st.c1 * Xi + (st.c2 * dt) * dq
            if st.acc_in >= 0 and st.c0 != 0.0:
                acc = acc + st.c0 * e.interior(e.pool[st.acc_in])
            acc = phys.finalize(acc, e.tens)
        out = st.a2 * dt * dq
        if st.a1 != 0.0:
            out = out + st.a1 * Qi
        if st.a0 != 0.0:
            out = out + st.a0 * Xi
        out = phys.finalize(out, e.tens)
        if st.acc_out >= 0:
            e.interior(e.pool[st.acc_out]).copy_(acc)
        e.interior(e.pool[st.out]).copy_(out)


class Engine:
    def __init__(self, physics: Physics, layout: TileLayout, rank: int = 0, grid: Optional[CubedSphereGrid] = None,
                 dtype=torch.float64, device="cpu", transport: Optional[Transport] = None, backend: str = "torch",
                 integrator: str = "ssprk3", dt: Optional[float] = None, cfl: Optional[float] = None, block=None):
        if physics.halo > layout.ng:
            raise ValueError(f"{physics.name} needs halo {physics.halo} > layout ng {layout.ng}")
        self.physics = physics
        self.layout = layout
        self.rank = rank
        self.grid = grid or CubedSphereGrid(layout.N)
        self.dtype = dtype
        self.device = torch.device(device)
        self.plan = layout.plan(rank)
        self.geo = RankGeometry(self.grid, layout, rank)
        self.tens: Dict[str, torch.Tensor] = physics.setup(self.geo, dtype, self.device)
        self.gmap = torch.as_tensor(self.plan.ghost_map, device=self.device)
        self.cmap = torch.as_tensor(self.plan.corner_map, device=self.device)
        self.integ: Integrator = get_integrator(integrator)
        F, S = physics.F, self.plan.S
        # padded storage, zero-initialised (corner ghost blocks are never written
        # nor read: see corner_slots / poison_corners)
        self.pool: List[torch.Tensor] = [torch.zeros((F, S), dtype=dtype, device=self.device) for _ in range(self.integ.nbuf)]
        self.halo_src = torch.as_tensor(self.plan.halo_src, dtype=torch.long, device=self.device)
        self.halo_dst = torch.as_tensor(self.plan.halo_dst, dtype=torch.long, device=self.device)
        self.transport = transport or NullTransport(self.plan, F, dtype, self.device)
        self.set_state(torch.as_tensor(physics.initial_state(self.geo), dtype=dtype))
        self.dt = float(dt) if dt is not None else (physics.max_dt(self.grid) if cfl is None else physics.max_dt(self.grid, cfl))
        self.time = 0.0
        self.step_count = 0
        self.backend = backend
        self.block = tuple(block) if block is not None else None   # None: ops.hip_compute.choose_block
        if backend == "torch":
            self.compute = TorchCompute(self)
        elif backend == "hip":
            from .ops.hip_compute import HipCompute
            self.compute = HipCompute(self)
        else:
            raise ValueError(f"unknown backend {backend!r}")

    # ---- state ------------------------------------------------------------
    @property
    def state(self) -> torch.Tensor:
        return self.pool[0]

    def interior(self, q: torch.Tensor) -> torch.Tensor:
        """[F, S] padded buffer -> [F, T, n, n] interior view."""
        return interior(q, self.plan.T, self.plan.n, self.plan.ng)

    def set_state(self, q: torch.Tensor) -> None:
        """q: [F, T, n, n] interior values (any device); refreshes the halos."""
        self.interior(self.pool[0]).copy_(q.reshape(self.physics.F, self.plan.T, self.plan.n, self.plan.n))
        self.refresh_halos(self.pool[0])

    def refresh_halos(self, q: torch.Tensor) -> None:
        """Fill the same-rank ghost slots of a padded buffer from their source
        cells (the HIP stages keep them current by pushing; needed after any
        external write of the state)."""
        if self.halo_src.numel():
            q[:, self.halo_dst] = q[:, self.halo_src]

    def tiles_view(self, q: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.interior(self.state if q is None else q)

    def corner_slots(self) -> torch.Tensor:
        """Flat padded-storage indices of the tile-corner ghost slots (both
        coordinates outside the tile) that no exchange writes: all but the
        carried panel-edge strip ends (``RankPlan.corner_map``).  At a cube
        corner three panels meet and the block has no single source.  The
        dimension-split stencils never read them (x-sweeps read ghost
        columns of the tile's own rows, y-sweeps ghost rows of its own
        columns); ``poison_corners`` makes that a checked property."""
        n, mg, T = self.plan.n, self.plan.ng, self.plan.T
        pw = n + 2 * mg
        c = torch.arange(pw)
        out = (c < mg) | (c >= n + mg)
        m2 = out[:, None] & out[None, :]
        idx = torch.nonzero(m2.reshape(-1)).reshape(-1)
        allc = (torch.arange(T)[:, None] * pw * pw + idx[None, :]).reshape(-1)
        from .parallel.layout import corner_xy
        cm = self.plan.corner_carried
        if cm.any():
            t, q, a, b = np.nonzero(cm)
            x, y = corner_xy(q, a, b, n)
            carried = torch.as_tensor((t * pw + y + mg) * pw + x + mg)
            allc = allc[~torch.isin(allc, carried)]
        return allc.to(self.device)

    def poison_corners(self) -> None:
        """Fill every corner ghost slot of every buffer with NaN: a stencil
        that ever reads one poisons the state (tests/test_numerics.py)."""
        idx = self.corner_slots()
        for b in self.pool:
            b[:, idx] = float("nan")

    # ---- stepping -----------------------------------------------------------
    canary = False   # debug race screen, HIP backend, eager only

    def stage_begin(self, st: Stage) -> None:
        if self.canary and self.backend == "hip":
            # every same-rank ghost slot of the output must be re-pushed this stage
            self.pool[st.out][:, self.halo_dst] = float("nan")
            if self.transport.recv.numel():
                self.transport.recv.fill_(float("nan"))
        self.transport.start(self.pool[st.Q])
        self.compute.stage(st, self.dt, None, part="interior")

    def stage_end(self, st: Stage) -> None:
        recv = self.transport.finish()
        if self.canary and self.backend == "hip" and recv is not None and recv.numel():
            if not bool(torch.isfinite(recv).all()):
                raise RuntimeError("canary: a remote ghost slot was not delivered by the exchange")
        self.compute.stage(st, self.dt, recv, part="boundary")
        if self.canary and self.backend == "hip":
            out = self.pool[st.out]
            bad = ~torch.isfinite(out[:, self.halo_dst])
            if bool(bad.any()):
                raise RuntimeError(f"canary: {int(bad.sum())} ghost slots not written by the stage kernel")

    def end_step(self) -> None:
        rot = self.integ.rotation
        self.pool = [self.pool[r] for r in rot]
        self.time += self.dt
        self.step_count += 1

    def step(self, nsteps: int = 1) -> None:
        for _ in range(nsteps):
            for st in self.integ.stages:
                self.stage_begin(st)
                self.stage_end(st)
            self.end_step()

    def diagnostics(self) -> Dict[str, float]:
        d = self.physics.diagnostics(self.tiles_view(), self.tens)
        return {k: float(v) for k, v in d.items()}

    def global_field(self, f: int = 0) -> np.ndarray:
        """Single-rank only: [6, N, N] float64 of field f."""
        assert self.layout.num_ranks == 1
        return assemble_global(self.layout, {0: self.tiles_view()[f].detach().cpu().numpy()})


class GraphStepper:
    """Capture `k` whole time steps (a multiple of the integrator's buffer
    period) of a GPU engine into one HIP graph and replay it: removes the host
    launch overhead that dominates small grids."""

    def __init__(self, engine: Engine, steps_per_graph: int = 10, warmup: bool = True):
        self.e = engine
        p = engine.integ.period
        self.k = max(p, ((steps_per_graph + p - 1) // p) * p)
        self.stream = torch.cuda.Stream(device=engine.device)
        t0, c0, pool0 = engine.time, engine.step_count, list(engine.pool)
        saved = [b.clone() for b in engine.pool]
        self.stream.wait_stream(torch.cuda.current_stream(engine.device))
        if warmup:
            with torch.cuda.stream(self.stream):
                engine.step(p)
        torch.cuda.current_stream(engine.device).wait_stream(self.stream)
        torch.cuda.synchronize(engine.device)
        engine.pool = pool0
        for b, s in zip(engine.pool, saved):
            b.copy_(s)
        torch.cuda.synchronize(engine.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            engine.step(self.k)
        engine.pool = pool0
        engine.time, engine.step_count = t0, c0
        self._pool0 = list(pool0)

    def _sync_pool(self) -> None:
        """The graph holds the construction-order buffer pointers; after an
        eager remainder rotated ``e.pool`` (period > 1), copy the buffers back
        into that order."""
        e = self.e
        if all(a is b for a, b in zip(e.pool, self._pool0)):
            return
        vals = [b.clone() for b in e.pool]
        for b, v in zip(self._pool0, vals):
            b.copy_(v)
        e.pool = list(self._pool0)

    def run(self, nsteps: int) -> None:
        e = self.e
        self._sync_pool()
        full, rem = divmod(nsteps, self.k)
        for _ in range(full):
            self.graph.replay()
        e.time += full * self.k * e.dt
        e.step_count += full * self.k
        if rem:
            e.step(rem)
            self._sync_pool()


def assemble_global(layout: TileLayout, tiles_by_rank: Dict[int, np.ndarray]) -> np.ndarray:
    """{rank: [T, n, n]} -> [6, N, N]."""
    N, n = layout.N, layout.n
    out = np.zeros((6, N, N))
    for r, arr in tiles_by_rank.items():
        for li, tid in enumerate(layout.rank_tiles[r]):
            f, I0, J0 = layout.tile_origin(tid)
            out[f, J0:J0 + n, I0:I0 + n] = arr[li]
    return out


class VirtualCluster:
    """All ranks of a layout in one process, stepped in lockstep (the analogue
    of the reference's CPU virtual devices, PY:64-68)."""

    def __init__(self, physics_factory, layout: TileLayout, **engine_kw):
        from .parallel.comm import VirtualHub
        self.layout = layout
        self.hub = VirtualHub()
        self.engines: List[Engine] = []
        for r in range(layout.num_ranks):
            phys = physics_factory()
            plan = layout.plan(r)
            dtype = engine_kw.get("dtype", torch.float64)
            dev = engine_kw.get("device", "cpu")
            tr = self.hub.transport(plan, phys.F, dtype, torch.device(dev))
            self.engines.append(Engine(phys, layout, r, transport=tr, **engine_kw))

    def step(self, nsteps: int = 1) -> None:
        for _ in range(nsteps):
            for st in self.engines[0].integ.stages:
                for e in self.engines:
                    e.stage_begin(st)
                for e in self.engines:
                    e.stage_end(st)
            for e in self.engines:
                e.end_step()

    def global_field(self, f: int = 0) -> np.ndarray:
        return assemble_global(self.layout, {e.rank: e.tiles_view()[f].detach().cpu().numpy() for e in self.engines})
