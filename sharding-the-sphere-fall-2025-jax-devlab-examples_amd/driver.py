"""Solver driver: the "JAXStream" pipeline of PDF s.6 (Geometry -> Initial
Conditions -> Solver -> {History, Restarts, Analysis}) on MI355X.

The reference shows only a method ``setup_sharding(self)`` of an unnamed class
holding ``self.config``, ``self.mesh`` and ``self.sharding`` (PY:19-85).
``Solver`` is that class:

    solver = Solver("config.yaml")      # or a dict / Config
    solver.setup_sharding()             # validation + banner, sets .mesh/.sharding
    solver.initialize()                 # grid, physics, per-rank engines, restore
    summary = solver.run(days=5)        # time loop, history, checkpoints, metrics

Execution modes (chosen from the config and the launch environment):

* ``single``  one device (GPU: fused HIP stage kernels + HIP-graph replay;
              CPU: PyTorch reference);
* ``virtual`` several ranks in one process, stepped in lockstep (the analogue
              of the reference's CPU virtual devices, PY:64-68; also works on
              one GPU);
* ``spmd``    one process per device under ``torchrun`` (WORLD_SIZE > 1):
              RCCL (backend "nccl") on GPUs, gloo on CPUs, bundled P2P halos.
"""
from __future__ import annotations

import math
import os
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .engine import Engine, GraphStepper, VirtualCluster, assemble_global
from .models.advection import Advection
from .models.base import limiter_code
from .models.diffusion import Diffusion
from .models.geometry import DAY, EARTH_RADIUS, CubedSphereGrid
from .models.swe import ShallowWater
from .parallel.comm import NativeBuffers, TorchDistTransport
from .parallel.layout import TileLayout
from .parallel.mesh import setup_sharding
from .utils import checkpoint as ckpt
from .utils.config import Config, default_case, load_config
from .utils.history import HistoryWriter, MetricsLogger


def make_physics(pc) -> Any:
    model = pc.model.lower()
    case = pc.case or default_case(model)
    lim = limiter_code(pc.limiter)
    if model == "swe":
        return ShallowWater(case, limiter=lim, alpha=pc.alpha)
    if model == "advection":
        return Advection(case, alpha=pc.alpha, limiter=lim)
    if model == "diffusion":
        return Diffusion(kappa=pc.kappa, case=case)
    raise ValueError(f"unknown physics model {pc.model!r}")


class _HostQueue:
    """Host work of the run loop, in submission order: ``append((event,
    work))`` runs ``work()`` once ``event`` (a CUDA event, or None) has
    completed; threaded, on one background thread, else inline at ``drain``."""

    def __init__(self, threaded: bool):
        self._items: List[Any] = []
        self._ex = None
        if threaded:
            from concurrent.futures import ThreadPoolExecutor
            self._ex = ThreadPoolExecutor(max_workers=1, thread_name_prefix="stsp-io")

    def append(self, item) -> None:
        ev, work = item
        if self._ex is None:
            self._items.append(item)
            return

        def job():
            if ev is not None:
                ev.synchronize()
            work()
        self._items.append(self._ex.submit(job))

    def __len__(self) -> int:
        return len(self._items)

    def drain(self, block: bool = False) -> None:
        """Finish the completed items (all of them when ``block``); a failed
        background item raises here."""
        while self._items:
            it = self._items[0]
            if self._ex is not None:
                if not block and not it.done():
                    return
                self._items.pop(0).result()
                continue
            ev, work = it
            if not block and ev is not None and not ev.query():
                return
            self._items.pop(0)
            if ev is not None:
                ev.synchronize()
            work()

    def close(self) -> None:
        self.drain(block=True)
        if self._ex is not None:
            self._ex.shutdown(wait=True)
            self._ex = None

    def clear(self) -> None:
        """Drop what has not run yet (recovery); a running item completes."""
        for it in self._items:
            if self._ex is not None:
                it.cancel()
        if self._ex is not None:
            for it in self._items:
                if not it.cancelled():
                    it.exception()
        self._items = []


class Solver:
    def __init__(self, config=None, verbose: bool = True):
        self.cfg: Config = load_config(config)
        self.config: Dict[str, Any] = self.cfg.to_dict()
        self.verbose = verbose
        self.mesh = None
        self.sharding = None
        self.engines: List[Engine] = []
        self.cluster: Optional[VirtualCluster] = None
        self.runner = None            # NativeStepper (GPU) once stepping starts
        self.fused = None             # ops/fused.py::FusedKernel when the runner steps with it
        self.xgmi = None
        self._ipc = None
        self._nccl = None
        self.comm = "local"
        self.mode = None
        self.world, self.rank = 1, 0

    # ---- setup ------------------------------------------------------------
    def setup_sharding(self) -> None:
        self.mesh, self.sharding = setup_sharding(self.config, verbose=self.verbose and self._is_root())

    def _is_root(self) -> bool:
        return int(os.environ.get("RANK", "0")) == 0

    def _log(self, *a) -> None:
        if self.verbose and self.rank == 0:
            print(*a, flush=True)

    def initialize(self) -> None:
        if self.sharding is None:
            self.setup_sharding()
        c = self.cfg
        nd = c.parallelization.num_devices
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        gpu = c.parallelization.device_type == "gpu"
        if gpu and not torch.cuda.is_available():
            raise RuntimeError("device_type 'gpu' requested but no GPU is visible (use device_type: cpu)")
        if self.world > 1:
            if self.world != nd:
                raise ValueError(f"launched with {self.world} processes but num_devices = {nd}")
            self.mode = "spmd"
            import torch.distributed as dist
            # STSP_SHARE_GPU=1: every rank on cuda:0 with a gloo group (functional
            # rehearsal of the multi-GPU paths on a one-GPU machine)
            share = os.environ.get("STSP_SHARE_GPU") == "1"
            device = torch.device(f"cuda:{0 if share else local}") if gpu else torch.device("cpu")
            if gpu:
                torch.cuda.set_device(device)
            if not dist.is_initialized():
                if gpu and not share:
                    dist.init_process_group("nccl", device_id=device)
                else:
                    dist.init_process_group("gloo")
        else:
            self.mode = "single" if nd == 1 else "virtual"
            device = torch.device("cuda:0") if gpu else torch.device("cpu")
        self.device = device
        backend = c.runtime.backend
        if backend == "auto":
            backend = "hip" if device.type == "cuda" else "torch"
        self.backend = backend
        dtype = {"float64": torch.float64, "fp64": torch.float64, "float32": torch.float32,
                 "fp32": torch.float32}[c.grid.dtype]
        self.dtype = dtype
        N, t = c.grid.N, c.parallelization.tiles_per_edge
        phys0 = make_physics(c.physics)
        # PPM reads three ghost layers: widen the halo if the config asks for fewer
        self.layout = TileLayout(N, t, nd, ng=max(c.grid.halo, phys0.halo), owner=self.sharding.owner)
        self.grid = self._geometry_stage(N, c.grid.radius or EARTH_RADIUS)
        dt = c.time.dt or (phys0.max_dt(self.grid, c.time.cfl) if c.time.cfl else phys0.max_dt(self.grid))
        kw = dict(grid=self.grid, dtype=dtype, device=device, backend=backend, integrator=c.time.integrator, dt=dt)
        if c.runtime.block:
            kw["block"] = tuple(c.runtime.block)
        if self.mode == "virtual":
            self.cluster = VirtualCluster(lambda: make_physics(c.physics), self.layout, **kw)
            self.engines = list(self.cluster.engines)
        elif self.mode == "spmd":
            comm = c.runtime.comm
            if comm == "auto":
                # GPUs: the native runtime with the direct xGMI exchange
                comm = "xgmi" if (backend == "hip" and c.runtime.graph and not c.runtime.canary) else "torch"
            if comm in ("xgmi", "rccl", "ipc") and backend != "hip":
                raise ValueError(f"runtime.comm = {comm} needs the HIP backend")
            self.comm = comm
            if comm in ("xgmi", "rccl", "ipc"):
                tr = NativeBuffers(self.layout.plan(self.rank), phys0.F, dtype, device)
            else:
                tr = TorchDistTransport(self.layout.plan(self.rank), phys0.F, dtype, device,
                                        staged=(comm == "staged"))
            self.engines = [Engine(phys0, self.layout, self.rank, transport=tr, **kw)]
        else:
            self.engines = [Engine(phys0, self.layout, 0, **kw)]
        for e in self.engines:
            e.canary = c.runtime.canary
        self.dt = dt
        self.physics = phys0
        self.fields = list(phys0.fields)
        self._log(f"Initialized {phys0.name} ({getattr(phys0, 'case', '')}) C{N}, {self.mode} mode, "
                  f"backend={backend}, dtype={c.grid.dtype}, dt={dt:.3f} s, integrator={c.time.integrator}")
        if c.io.initial_condition and not c.io.restore:
            self._initial_condition_stage(c.io.initial_condition)
        if c.io.restore:
            path = c.io.restore
            if path == "latest":
                path = ckpt.latest_checkpoint(self.checkpoint_root())
            if path:
                self.restore_checkpoint(path)

    # ---- pipeline stages: Geometry and Initial Conditions through zarr (PDF s.6) ----
    def _geometry_stage(self, N: int, radius: float) -> CubedSphereGrid:
        """Read the grid from ``io.geometry`` when that zarr group exists, else
        compute it and (rank 0) write it there."""
        path = self.cfg.io.geometry
        if path and os.path.exists(os.path.join(path, ".zgroup")):
            g = CubedSphereGrid.load_zarr(path, N=N, radius=radius)
            self._log(f"Geometry: read C{N} grid from {path}")
            return g
        g = CubedSphereGrid(N, radius)
        if path:
            if self.rank == 0:
                g.save_zarr(path)
                self._log(f"Geometry: wrote C{N} grid to {path}")
            self._barrier()
        return g

    def _initial_condition_stage(self, path: str) -> None:
        """Read the initial state [F, 6, N, N] from ``io.initial_condition``
        when that zarr group exists, else (rank 0) write the analytic initial
        condition the engines were built with.  Partition-independent, like
        checkpoints."""
        from .utils import zarr_lite
        if os.path.exists(os.path.join(path, ".zgroup")):
            attrs = zarr_lite.read_attrs(path)
            if int(attrs["N"]) != self.layout.N or list(attrs["fields"]) != list(self.fields):
                raise ValueError(f"{path}: initial condition is C{attrs['N']} {attrs['fields']}, "
                                 f"run is C{self.layout.N} {self.fields}")
            # the state must belong to this physics and case: TC2 and TC5 share the
            # SWE fields but not the topography the engines were built with
            want = {"physics": self.physics.name, "case": getattr(self.physics, "case", None)}
            for k, v in want.items():
                if k in attrs and attrs[k] != v:
                    raise ValueError(f"{path}: initial condition was written for {k} {attrs[k]!r}, "
                                     f"the run is {k} {v!r} (remove the file or fix io.initial_condition)")
            glob = np.stack([zarr_lite.read_array(path, f) for f in self.fields])
            for e in self.engines:
                loc = np.stack([e.geo.gather_global(glob[k]) for k in range(len(self.fields))])
                e.set_state(torch.as_tensor(loc, dtype=self.dtype))
            self._log(f"Initial conditions: read {path}")
            return
        g = self.gather_global()
        if self.rank == 0:
            zarr_lite.create_group(path, attrs={"N": self.layout.N, "fields": self.fields,
                                                "physics": self.physics.name,
                                                "case": getattr(self.physics, "case", None), "time": self.time})
            for k, f in enumerate(self.fields):
                zarr_lite.write_array(path, f, g[k], chunks=(1, self.layout.N, self.layout.N))
            self._log(f"Initial conditions: wrote {path}")
        self._barrier()

    # ---- state access ---------------------------------------------------------
    @property
    def time(self) -> float:
        return self.engines[0].time

    @property
    def step_count(self) -> int:
        return self.engines[0].step_count

    def local_values(self) -> Dict[int, np.ndarray]:
        """{rank: [F, T_local, n, n]} for the engines of this process."""
        return {e.rank: e.tiles_view().detach().cpu().double().numpy() for e in self.engines}

    def gather_global(self) -> Optional[np.ndarray]:
        """[F, 6, N, N] on rank 0 (None elsewhere)."""
        F = len(self.fields)
        vals = self.local_values()
        if self.mode == "spmd":
            import torch.distributed as dist
            objs = [None] * self.world
            dist.all_gather_object(objs, vals)
            vals = {}
            for o in objs:
                vals.update(o)
            if self.rank != 0:
                return None
        return np.stack([assemble_global(self.layout, {r: v[f] for r, v in vals.items()}) for f in range(F)])

    def global_field(self, name_or_index=0) -> Optional[np.ndarray]:
        f = self.fields.index(name_or_index) if isinstance(name_or_index, str) else name_or_index
        g = self.gather_global()
        return None if g is None else g[f]

    def _allreduce(self, vals: Dict[str, float], op: str = "sum") -> Dict[str, float]:
        if self.mode != "spmd":
            return vals
        import torch.distributed as dist
        keys = sorted(vals)
        t = torch.tensor([vals[k] for k in keys], dtype=torch.float64,
                         device=self.device if self.device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MIN)
        return dict(zip(keys, t.tolist()))

    def diagnostics(self) -> Dict[str, float]:
        tot: Dict[str, float] = {}
        for e in self.engines:
            for k, v in e.diagnostics().items():
                tot[k] = tot.get(k, 0.0) + v
        return self._allreduce(tot)

    def error_norms(self) -> Optional[Dict[str, float]]:
        """Williamson l1 / l2 / linf of field 0 against the case's true
        solution at the current time (TC1, TC2, lake at rest), on rank 0;
        None where the case has no closed form (and on other ranks)."""
        from .models.errors import williamson_norms
        exact = getattr(self.physics, "exact", None)
        h = self.global_field(0)
        if exact is None or h is None:
            return None
        ht = exact(self.grid, self.time)
        if ht is None:
            return None
        return williamson_norms(h, ht, self.grid.areas())

    def all_finite(self) -> bool:
        if self.runner is not None:
            self.runner.check()      # direct xGMI exchange: raises on a halo poll timeout
        ok = float(all(bool(torch.isfinite(e.tiles_view()).all()) for e in self.engines))
        return self._allreduce({"ok": ok}, op="min")["ok"] > 0.5

    # ---- stepping ---------------------------------------------------------------
    def _use_native(self) -> bool:
        """Step through the C++ runtime (ops/native_runtime.py): one GPU with
        graph replay, or SPMD GPUs with the direct xGMI / RCCL exchange."""
        c = self.cfg.runtime
        if self.backend != "hip" or c.canary:
            return False
        if self.mode == "single":
            return c.graph
        return self.mode == "spmd" and self.comm in ("xgmi", "rccl", "ipc")

    def _fused_plan(self, chunks):
        """(use the fused step, steps per launch) for this run.  The fused
        SSP-RK3 step (ops/fused.py) is the flagship path: one launch advances
        a rank by several steps (every block resident, in-launch hand-offs), the
        reference's "one compiled program" (PY:238-246; PDF s.10) driven from the
        solver (PDF s.6 pipeline).  auto: shallow water + SSP-RK3 + PLR, one GPU
        or SPMD ranks with the direct xGMI exchange, and at most two passes of
        blocks over the CUs (one step per launch beyond one pass)."""
        from .ops.fused import fused_block, fused_supported, rank_cus
        c = self.cfg.runtime
        e = self.engines[0]
        if c.fused == "off" or e.device.type != "cuda":
            return False, 1
        # one GPU, or SPMD ranks with the direct xGMI exchange (the ring inside
        # the fused kernel); auto takes the multi-rank fused step when every
        # block of the rank's share is resident (checked below)
        if not (self.mode == "single" or (self.mode == "spmd" and self.comm == "xgmi")):
            if c.fused == "on":
                raise ValueError(f"runtime.fused = on needs one GPU or the xgmi exchange (mode {self.mode}, "
                                 f"comm {self.comm})")
            return False, 1
        why = fused_supported(e)
        if why:
            if c.fused == "on":
                raise ValueError(why)
            return False, 1
        cus = rank_cus(e.device)
        B = fused_block(e.plan.n, len(e.plan.tiles), cus)
        nb = len(e.plan.tiles) * (e.plan.n // B) ** 2
        if c.fused == "auto" and nb > (2 * cus if self.mode == "single" else cus):
            return False, 1
        if nb > cus:
            return True, 1                     # one step per launch (blocks not all resident)
        spl = c.steps_per_launch
        if spl <= 0:
            # the longest even launch dividing EVERY chunk length of the run
            # (each launch boundary costs ~18 us of ramp, profiles/r4_spl/); a
            # run whose chunks share no even divisor launches its longest even
            # part per chunk, the rest through the remainder path (its
            # descriptors are built and primed by prepare())
            lens = [max(1, int(k)) for k in (chunks if isinstance(chunks, (list, tuple)) else [chunks])]
            g = 0
            for k in lens:
                g = math.gcd(g, k)
            divs = [s for s in range(2, 513, 2) if g % s == 0]
            k0 = min(lens)
            spl = max(divs) if divs else (min(512, k0 - k0 % 2) if k0 >= 2 else 1)
        if spl > 1 and spl % 2:
            raise ValueError("runtime.steps_per_launch must be even")
        return True, spl

    def _make_runner(self, chunks=(20,)):
        from .ops.native_runtime import NativeStepper, create_nccl_comm
        e = self.engines[0]
        c = self.cfg.runtime
        use_fused, spl = self._fused_plan(list(chunks))
        self.fused = None
        if use_fused:
            from .ops.fused import FusedKernel, fused_block, rank_cus
            cus = rank_cus(e.device)
            try:
                fk = FusedKernel(e, B=fused_block(e.plan.n, len(e.plan.tiles), cus))   # collective with several ranks
            except RuntimeError as exc:
                if self.mode != "spmd":
                    raise
                # the ring setup raised on every rank alike: the stage-kernel op
                # list with the next transport of the chain
                self._log(f"Runtime: fused xGMI step unavailable ({exc}); falling back")
                self.comm = "ipc"
                fk = None
            if fk is not None:
                self.fused = fk
                self.xgmi = fk if self.mode == "spmd" else None
                self._log(f"Runtime: fused SSP-RK3 step, {fk.plan.nb} blocks of {fk.plan.B}x{fk.plan.B}, "
                          f"{spl} step(s) per launch, " + ("direct launches" if self.mode == "single" else "graph replay"))
                return NativeStepper(e, use_graph=True, steps_per_graph=c.steps_per_graph, fused=fk,
                                     steps_per_launch=spl, direct=self.mode == "single")
        if self.mode == "single" and c.march3 != "off":
            from .ops.march3 import March3Step, march3_unsupported, march3_wanted
            why = march3_unsupported(e)
            if c.march3 == "on" and why:
                raise ValueError(f"runtime.march3 = on: {why}")
            if c.march3 == "on" or march3_wanted(e):
                m3 = March3Step(e, rows=c.march3_rows)
                self._log(f"Runtime: pipelined SSP-RK3 march ({m3.ncs} strips x {m3.nrs} segments per tile, "
                          f"{m3.band.numel()} band blocks), graph replay")
                self.xgmi = self._ipc = None
                return NativeStepper(e, use_graph=c.graph, steps_per_graph=c.steps_per_graph, march3=m3)
        xg = nc = ipc = None
        if self.mode == "spmd":
            # transport chain between GPUs: direct xGMI rings -> IPC copy kernel
            # (graph-captured) -> RCCL (eager).  A setup that fails raises on
            # every rank alike (IpcRing agrees on every step), so all ranks
            # move down the chain together.
            order = ["xgmi", "ipc", "rccl"]
            chain = order[order.index(self.comm):] if self.comm in order else [self.comm]
            for k, cm in enumerate(chain):
                try:
                    if cm == "xgmi":
                        from .ops.xgmi import XgmiHalo
                        xg = XgmiHalo(e)
                    elif cm == "ipc":
                        from .ops.native_runtime import IpcExchange
                        ipc = IpcExchange(e, IpcExchange.slots_for(e))        # collective (IPC handles)
                    elif cm == "rccl":
                        if self._nccl is None:
                            self._nccl = create_nccl_comm(self.rank, self.world, self.device.index or 0)
                        nc = self._nccl
                    self.comm = cm
                    break
                except RuntimeError as exc:
                    if k == len(chain) - 1:
                        raise
                    self._log(f"Runtime: {cm} exchange unavailable ({exc}); falling back to {chain[k + 1]}")
        self.xgmi = xg
        self._ipc = ipc
        return NativeStepper(e, nccl_comm=nc, use_graph=c.graph, steps_per_graph=c.steps_per_graph, xgmi=xg,
                             ipc=ipc)

    def close(self) -> None:
        """Release the step runner and the exchange rings explicitly.  With
        several ranks this is collective (every rank calls it, as the run
        script does at the end): the rings' close joins a group barrier, which
        a garbage-collection finalizer must not do."""
        if self.runner is not None:
            self.runner.close()
            self.runner = None
        seen = set()
        for obj in (self.xgmi, self.fused, getattr(self, "_ipc", None)):
            if obj is not None and id(obj) not in seen and hasattr(obj, "close"):
                seen.add(id(obj))
                obj.close()
        self.xgmi = self.fused = self._ipc = None

    def step(self, nsteps: int = 1) -> None:
        if nsteps <= 0:
            return
        if self.mode == "virtual":
            self.cluster.step(nsteps)
        elif self._use_native():
            if self.runner is None:
                self.runner = self._make_runner()
            self.runner.run(nsteps)
        else:
            self.engines[0].step(nsteps)

    def _sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # ticks per step at the run's initial dt: the watchdog halves dt at most
    # three times, so every interval stays a whole number of steps
    _SUB = 8

    def run(self, nsteps: Optional[int] = None, days: Optional[float] = None) -> Dict[str, Any]:
        """Advance ``nsteps`` steps (or ``days``) of the run's initial dt.

        The loop is graph-aware: history / checkpoint / metrics / watchdog
        intervals cut the run into equal chunks, the native runner records one
        graph of that chunk length (plus the final remainder) before the clock
        starts, and every chunk is one graph replay.  History snapshots and
        metrics are copied device -> pinned host memory on the stepping stream
        and written out while the next chunk runs; the watchdog's finite-check
        is read one chunk late (single-process modes).  The summary reports
        the stepping throughput without setup (``setup_s``: graph capture and
        first replay), plus the host time of each phase (``phase_s``; each phase
        is also a roctx range).

        Watchdog recovery restores a checkpoint, halves the *current* dt and
        continues to the same simulated end time; history frames are indexed by
        simulated time, so replayed intervals overwrite their frames.
        """
        from .utils.tracing import PhaseTimes
        if not self.engines:
            self.initialize()
        c = self.cfg
        if nsteps is None:
            days = days if days is not None else c.time.days
            if days is not None:
                nsteps = int(math.ceil(days * DAY / self.dt - 1e-9))
            else:
                nsteps = c.time.nsteps or 1
        io = c.io
        out = io.output_dir
        ph = PhaseTimes()
        SUB = self._SUB
        dt0, t0 = self.dt, self.time
        end = nsteps * SUB
        level = 0                               # dt = dt0 / 2**level

        def pos() -> int:
            return int(round((self.time - t0) / dt0 * SUB))

        iv = {"history": io.history_interval, "checkpoint": io.checkpoint_interval,
              "metrics": io.metrics_interval, "watchdog": c.runtime.watchdog_interval}
        iv = {k: v * SUB for k, v in iv.items() if v > 0}
        hist = None
        if "history" in iv:
            n_out = nsteps // io.history_interval + 1
            hpath = os.path.join(out, "history.zarr")
            if self.rank == 0:
                os.makedirs(out, exist_ok=True)
                HistoryWriter(hpath, self.fields, self.layout.N, self.layout.n, n_out,
                              attrs={"config": self.config}, frame_chunks=self.mode != "spmd")
            self._barrier()
            hist = HistoryWriter(hpath, self.fields, self.layout.N, self.layout.n, n_out, create=False)
        metrics = MetricsLogger(os.path.join(out, "metrics.jsonl") if "metrics" in iv else None,
                                enabled=self.rank == 0)
        cells = 6 * self.layout.N ** 2
        gpu = self.device.type == "cuda"
        deferred = gpu and self.mode != "spmd"
        # (event, host work) done while the next chunks run: on a GPU by one
        # background thread (zarr / JSONL / checkpoint writes release the GIL),
        # so the loop keeps the launch queue full (a history frame's ~100 tile
        # files took ~10 ms of GPU idle per frame when written in the loop)
        pending = _HostQueue(threaded=deferred)

        def drain(block: bool = False) -> None:
            pending.drain(block)

        def chunk_at(p: int, step_ticks: int) -> int:
            nxt = min([(p // v + 1) * v for v in iv.values()] + [end])
            return max(1, (nxt - p) // step_ticks)

        # ---- setup: graphs for the chunk lengths this run replays ------------------
        with ph("setup"):
            if ("checkpoint" in iv and "watchdog" in iv
                    and self.step_count not in ckpt.list_checkpoints(self.checkpoint_root())):
                self.save_checkpoint()      # the watchdog can always roll back to the run's start
            if hist is not None:
                self._snapshot_history(hist, 0, pending, async_copy=False)
                drain(block=True)
            if self._use_native() and nsteps > 0:
                lens, p, it = [], 0, 0
                while p < end and it < 100000:        # the chunk sequence of a run without recovery
                    k = chunk_at(p, SUB)
                    if k not in lens:
                        lens.append(k)
                    p += k * SUB
                    it += 1
                if self.runner is None:
                    self.runner = self._make_runner(chunks=lens)
                per = self.runner.period
                self.runner.graph_periods = max(1, min(max(lens), 512) // per)
                for k in lens[:8]:
                    self.runner.prepare(k)      # chunks shorter than a period: their remainder launch
            if deferred and ("watchdog" in iv or "metrics" in iv):
                self._warm_checks()
            self._sync()
        wall0 = time.perf_counter()
        recoveries = 0
        done = 0
        self._wd_pending = None
        while True:
            p = pos()
            if p >= end:
                break
            st = SUB >> level
            chunk = chunk_at(p, st)
            with ph("step"):
                self.step(chunk)
            done += chunk
            drain()
            p = pos()
            due = {k for k, v in iv.items() if p % v == 0 or p >= end}
            ok, checked = True, False
            if "watchdog" in due:
                with ph("watchdog"):
                    sync_check = not (deferred and "checkpoint" not in due and p < end)
                    ok = self._watchdog(pending, not sync_check)
                    checked = sync_check
            if ok and "checkpoint" in due and p % iv["checkpoint"] == 0 and "watchdog" in iv and not checked:
                # a checkpoint between watchdog intervals: resolve the deferred
                # check and test the state itself, so no checkpoint ever holds a
                # state the watchdog would reject
                with ph("watchdog"):
                    drain(block=True)
                    ok = self._watchdog(pending, False)
            if not ok:
                drain(block=True)                   # checkpoints still being written
                saved = [s for s in ckpt.list_checkpoints(self.checkpoint_root())]
                if recoveries < 3 and saved:
                    recoveries += 1
                    pending.clear()
                    self._wd_pending = None
                    # go back further on each repeated failure (recent checkpoints may
                    # already hold a growing instability)
                    last = ckpt.step_dir(self.checkpoint_root(), saved[-min(recoveries, len(saved))])
                    dt_cur = self.dt
                    self._log(f"watchdog: non-finite state at step {self.step_count}; restarting from {last} "
                              f"with dt/2")
                    self.restore_checkpoint(last)
                    level += 1
                    self.set_dt(dt_cur * 0.5)
                    if abs(self.dt * (1 << level) - dt0) > 1e-9 * dt0:
                        self.set_dt(dt0 / (1 << level))
                    continue
                raise FloatingPointError(f"non-finite state detected at step {self.step_count}")
            if hist is not None and "history" in due and p % iv["history"] == 0:
                with ph("history"):
                    self._snapshot_history(hist, p // iv["history"], pending, async_copy=deferred)
            if "checkpoint" in due and p % iv["checkpoint"] == 0:
                with ph("checkpoint"):
                    if deferred:
                        self._checkpoint_async(pending)
                    else:
                        drain(block=True)
                        self.save_checkpoint()
            if "metrics" in due:                 # every interval and the end of the run
                with ph("metrics"):
                    self._snapshot_metrics(metrics, pending, deferred, cells, done, wall0, p)
        with ph("drain"):
            self._sync()
            pending.close()
            if self.runner is not None:
                # a producer wait or xGMI poll that timed out sets the kernel's
                # error word and the kernel carries on with stale cells: never
                # report such a run
                self.runner.check()
        wall = time.perf_counter() - wall0
        summary = {"steps": nsteps, "steps_run": done, "wall_s": wall, "setup_s": ph.times.get("setup", 0.0),
                   "sim_days": self.time / DAY,
                   "cell_updates_per_s": cells * done / max(wall, 1e-12),
                   "sim_days_per_day": ((self.time - t0) / DAY) / max(wall / DAY, 1e-30),
                   "recoveries": recoveries, "dt_final": self.dt,
                   "graph_steps": (self.runner.stats["graph_steps"] if self.runner is not None else 0),
                   "runtime": ("fused" if getattr(self, "fused", None) is not None else
                               "native" if self.runner is not None else "eager"),
                   "fused_direct_steps": (self.runner.stats["direct_steps"] if self.runner is not None else 0),
                   "kernel_launches": (self.runner.stats["launches"] if self.runner is not None else 0),
                   "phase_s": dict(ph.times)}
        summary.update(self.diagnostics())
        norms = self.error_norms()
        if norms is not None:
            summary.update({f"err_{k}": v for k, v in norms.items()})
        self._log(f"Run complete: {done} steps, {summary['sim_days']:.3f} days, "
                  f"{summary['cell_updates_per_s']:.3e} cell-updates/s (setup {summary['setup_s']:.3f} s excluded)")
        return summary

    # ---- run-loop helpers ----------------------------------------------------------
    def _snapshot_history(self, hist: HistoryWriter, k: int, pending: List[Any], async_copy: bool) -> None:
        """History frame k: the interior values are copied to host memory on
        the stepping stream; the zarr chunks are written when the copy is done
        (``pending``), i.e. while the next chunk steps."""
        t, sc = self.time, self.step_count
        snaps = []
        for e in self.engines:
            v = e.tiles_view().detach()
            if async_copy:
                h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                h.copy_(v, non_blocking=True)
            else:
                h = v.cpu()
            snaps.append((e.plan.tiles, h))
        ev = None
        if async_copy:
            ev = torch.cuda.Event()
            ev.record()

        def work():
            parts = [(list(tiles), h.double().numpy()) for tiles, h in snaps]
            if hist.frame_chunks and len(parts) > 1:      # every engine of this process in one frame
                parts = [(sum((p_[0] for p_ in parts), []), np.concatenate([p_[1] for p_ in parts], 1))]
            for tiles, arr in parts:
                hist.write_tiles(k, tiles, self.layout.tile_origin, arr)
            if self.rank == 0:
                hist.write_time(k, t, sc)
        pending.append((ev, work))

    def _snapshot_metrics(self, metrics: MetricsLogger, pending: List[Any], deferred: bool, cells: int,
                          done: int, wall0: float, p: int) -> None:
        rec = dict(step=self.step_count, time_s=self.time, sim_days=self.time / DAY, dt=self.dt)
        wall = time.perf_counter() - wall0
        rec["cell_updates_per_s"] = cells * done / max(wall, 1e-12)
        if not deferred:
            metrics.log(**rec, **self.diagnostics())
            return
        keys, vals = [], []
        for e in self.engines:
            for k, v in e.physics.diagnostics(e.tiles_view(), e.tens).items():
                keys.append(k)
                vals.append(v.reshape(()).to(torch.float64))
        dev = torch.stack(vals)
        h = torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True)
        h.copy_(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()

        def work():
            tot: Dict[str, float] = {}
            for k, v in zip(keys, h.tolist()):
                tot[k] = tot.get(k, 0.0) + v
            metrics.log(**rec, **tot)
        pending.append((ev, work))

    def _warm_checks(self) -> None:
        """Run the watchdog and metrics reductions once before the clock
        starts.  Their first use in a process loads the kernels' code objects
        and the first pinned host blocks: measured on a 2-day C48 run
        (tools/run_phase_probe.py, profiles/r2_run_phases) that cost ~15 ms
        and took the run from 14.6 to 156 us/step with only the watchdog on."""
        flag = torch.stack([torch.isfinite(e.tiles_view()).all() for e in self.engines]).all()
        vals = [v.reshape(()).to(torch.float64) for e in self.engines
                for v in e.physics.diagnostics(e.tiles_view(), e.tens).values()]
        hf = torch.empty((), dtype=torch.bool, pin_memory=True)
        hf.copy_(flag, non_blocking=True)
        hv = torch.empty((len(vals),), dtype=torch.float64, pin_memory=True)
        hv.copy_(torch.stack(vals), non_blocking=True)
        torch.cuda.current_stream().synchronize()

    def _watchdog(self, pending: List[Any], deferred: bool) -> bool:
        """True while the state is finite.  Deferred (single process): the
        check of this interval is queued and the previous interval's result is
        returned, so the host never waits for the GPU here (a failure is seen
        one interval late; checkpoints drain the queue first, so a checkpoint
        never holds a state the watchdog has not passed)."""
        if not deferred:
            prev = getattr(self, "_wd_pending", None)
            self._wd_pending = None
            ok = self.all_finite()
            if prev is not None:
                ok = self._wd_result(prev) and ok
            return ok
        # [finite, no kernel error word set]: the error words of the fused step's
        # producer waits and the xGMI polls travel in the same pinned copy, so a
        # timed-out wait (the kernel then computes on stale cells) is seen one
        # interval late like a non-finite state, and raises
        finite = torch.stack([torch.isfinite(e.tiles_view()).all() for e in self.engines]).all()
        errs = self.runner.err_words() if self.runner is not None else []
        clean = torch.stack([(w[0] == 0) for w in errs]).all() if errs else torch.ones_like(finite)
        h = torch.empty(2, dtype=torch.bool, pin_memory=True)
        h.copy_(torch.stack([finite, clean]), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        prev = getattr(self, "_wd_pending", None)
        self._wd_pending = (ev, h)
        if prev is None:
            return True
        return self._wd_result(prev)

    def _wd_result(self, prev) -> bool:
        """Finite flag of a deferred watchdog copy; raises if a kernel error
        word was set (not a numerical failure: no rollback)."""
        prev[0].synchronize()
        if not bool(prev[1][1].item()):
            self.runner.check()
            raise RuntimeError("kernel error word set during the run")
        return bool(prev[1][0].item())

    def set_dt(self, dt: float) -> None:
        self.dt = dt
        for e in self.engines:
            e.dt = dt
        if self.runner is not None:
            self.runner.set_dt(dt)   # graphs bake dt in: the runner re-records

    def _barrier(self) -> None:
        if self.mode == "spmd":
            import torch.distributed as dist
            dist.barrier()

    def _write_history(self, hist: HistoryWriter, k: int) -> None:
        parts = [(list(e.plan.tiles), e.tiles_view().detach().cpu().double().numpy()) for e in self.engines]
        if hist.frame_chunks and len(parts) > 1:
            parts = [(sum((p_[0] for p_ in parts), []), np.concatenate([p_[1] for p_ in parts], 1))]
        for tiles, arr in parts:
            hist.write_tiles(k, tiles, self.layout.tile_origin, arr)
        if self.rank == 0:
            hist.write_time(k, self.time, self.step_count)

    def _checkpoint_async(self, pending: "_HostQueue") -> None:
        """Checkpoint of the current state without stopping the GPU (single
        process): the interior values are copied to pinned host memory on the
        stepping stream and the background writer commits the step directory
        once the copy is done (in order with the history frames before it)."""
        root = self.checkpoint_root()
        step, t, dt = self.step_count, self.time, self.dt
        snaps = []
        for e in self.engines:
            v = e.tiles_view().detach()
            h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
            h.copy_(v, non_blocking=True)
            snaps.append((e.plan.tiles, h))
        ev = torch.cuda.Event()
        ev.record()

        def work():
            self._write_checkpoint(root, step, t, dt, [(tiles, h.double().numpy()) for tiles, h in snaps])
        pending.append((ev, work))

    def _write_checkpoint(self, root: str, step: int, t: float, dt: float, parts) -> str:
        d = ckpt.step_dir(root, step)
        meta = {"step": step, "time": t, "dt": dt, "N": self.layout.N,
                "tiles_per_edge": self.layout.t, "num_ranks": self.layout.num_ranks,
                "owner": self.layout.owner, "fields": self.fields, "dtype": self.cfg.grid.dtype,
                "integrator": self.cfg.time.integrator, "physics": self.physics.name,
                "config": self.config, "format": "stsphere-ckpt-v1"}
        ckpt.begin(root, step, meta, self.fields, self.layout.N, self.layout.n, np.float64)
        for tiles, arr in parts:
            ckpt.write_tiles(d, self.fields, tiles, self.layout.tile_origin, arr, self.layout.n)
        ckpt.commit(d)
        ckpt.prune(root, self.cfg.io.keep_checkpoints)
        return d

    # ---- checkpoint / restart ------------------------------------------------------
    def checkpoint_root(self) -> str:
        return self.cfg.io.checkpoint_dir or os.path.join(self.cfg.io.output_dir, "checkpoints")

    def save_checkpoint(self, root: Optional[str] = None) -> str:
        root = root or self.checkpoint_root()
        self._sync()
        step = self.step_count
        d = ckpt.step_dir(root, step)
        if self.rank == 0:
            meta = {"step": step, "time": self.time, "dt": self.dt, "N": self.layout.N,
                    "tiles_per_edge": self.layout.t, "num_ranks": self.layout.num_ranks,
                    "owner": self.layout.owner, "fields": self.fields, "dtype": self.cfg.grid.dtype,
                    "integrator": self.cfg.time.integrator, "physics": self.physics.name,
                    "config": self.config, "format": "stsphere-ckpt-v1"}
            ckpt.begin(root, step, meta, self.fields, self.layout.N, self.layout.n, np.float64)
        self._barrier()
        for e in self.engines:
            ckpt.write_tiles(d, self.fields, e.plan.tiles, self.layout.tile_origin,
                             e.tiles_view().detach().cpu().double().numpy(), self.layout.n)
        self._barrier()
        if self.rank == 0:
            ckpt.commit(d)
            ckpt.prune(root, self.cfg.io.keep_checkpoints)
        self._barrier()
        return d

    def restore_checkpoint(self, path: str) -> None:
        meta = ckpt.read_meta(path)
        arrs = ckpt.read_fields(path, self.fields)
        if meta["N"] != self.layout.N:
            raise ValueError(f"checkpoint grid C{meta['N']} != configured C{self.layout.N}")
        glob = np.stack([arrs[f] for f in self.fields])           # [F,6,N,N]
        for e in self.engines:
            loc = np.stack([e.geo.gather_global(glob[k]) for k in range(len(self.fields))])
            e.set_state(torch.as_tensor(loc, dtype=self.dtype))
            e.time = float(meta["time"])
            e.step_count = int(meta["step"])
        if self.xgmi is not None:
            self.xgmi.prime()      # remote ghosts of the restored state (collective)
        self.set_dt(float(meta["dt"]))
        self._log(f"Restored {path} (step {meta['step']}, t = {meta['time'] / DAY:.4f} days, "
                  f"written by {meta['num_ranks']} rank(s), tiles_per_edge {meta['tiles_per_edge']})")
