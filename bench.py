#!/usr/bin/env python
"""Headline benchmark: cell-updates/s (whole node) of the cubed-sphere
shallow-water solver at C96 (BASELINE.json metric), plus simulated-days/day.

Flagship step: Williamson TC5 (zonal flow over a mountain; synthetic initial
condition, nothing downloaded), C96 = 6 x 96^2 cells, float64, SSP-RK3 (3 fused
gfx950 stage kernels per step), 24 tiles of 48^2 (tiles_per_edge = 2) so the
same decomposition runs on 1, 2, 4 and 8 GPUs (corner partition: a rank owns
the 3 face-quadrants around each cube vertex it holds).  Strong scaling: the
C96 problem is fixed as N grows.

    python bench.py                         # 1 GPU
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints one JSON line.  The timed region is exactly K full time steps
(every RK stage, every halo exchange) bracketed by barrier + synchronize; the
time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

BASELINE_CUPS = 2.6e8   # derived FV-PLR roofline cell-updates/s (900 GB/s device)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--tiles-per-edge", type=int, default=2)
    ap.add_argument("--case", default="tc5")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--integrator", default="ssprk3")
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--runtime", default="auto", choices=["auto", "persistent", "native", "graph", "eager"])
    ap.add_argument("--steps-per-graph", type=int, default=30)
    ap.add_argument("--comm", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="multi-GPU halo exchange of the native runtime: direct xGMI stores from the stage "
                         "kernels (graph-captured; default) or RCCL grouped send/recv (eager)")
    ap.add_argument("--partition", default="auto")
    ap.add_argument("--dt", type=float, default=None)
    ap.add_argument("--no-verify", action="store_true",
                    help="N > 1: skip the bitwise comparison with a one-GPU run after timing")
    return ap.parse_args()


def verify_single(a, phys, grid, dtype, device, dt, layout, tiles_by_rank, runtime, backend):
    """Max |difference| between the gathered multi-rank state and one rank
    stepping the same warmup + steps on this GPU (0.0 = bitwise equal)."""
    import numpy as np
    from stsphere.engine import Engine, assemble_global
    from stsphere.parallel.layout import TileLayout
    L1 = TileLayout(a.N, a.tiles_per_edge, 1, ng=layout.ng)
    ref = Engine(phys, L1, 0, grid=grid, dtype=dtype, device=device, backend=backend, integrator=a.integrator, dt=dt)
    total = a.warmup + a.steps
    if runtime == "native" and backend == "hip":
        from stsphere.ops.native_runtime import NativeStepper
        r = NativeStepper(ref, use_graph=True, steps_per_graph=a.steps_per_graph)
        r.run(total)
    else:
        ref.step(total)
    F = phys.F
    got = np.stack([assemble_global(layout, {r: t[f] for r, t in enumerate(tiles_by_rank)}) for f in range(F)])
    want = np.stack([ref.global_field(f) for f in range(F)])
    return float(np.abs(got - want).max())


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    from stsphere.engine import Engine, GraphStepper
    from stsphere.models.geometry import CubedSphereGrid, DAY
    from stsphere.models.swe import ShallowWater
    from stsphere.parallel.comm import NativeBuffers, TorchDistTransport
    from stsphere.parallel.layout import TileLayout

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus > 1 needs a torch.distributed launch (one process per GPU)")
    # STSP_SHARE_GPU=1: rehearsal mode, every rank on cuda:0 with a gloo group
    # (functional check of the multi-rank paths on a one-GPU box; not a benchmark)
    share = os.environ.get("STSP_SHARE_GPU") == "1"
    device = torch.device(f"cuda:{0 if share else local}") if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1:
        if device.type == "cuda" and not share:
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    dtype = torch.float64 if a.dtype == "fp64" else torch.float32
    layout = TileLayout(a.N, a.tiles_per_edge, world, ng=2, partition=a.partition)
    grid = CubedSphereGrid(a.N)
    phys = ShallowWater(a.case)
    backend = a.backend if device.type == "cuda" else "torch"
    runtime = a.runtime
    if runtime == "auto":
        runtime = "native" if (device.type == "cuda" and backend == "hip") else "eager"
    comm = a.comm if world > 1 else "none"
    if world > 1 and runtime != "native":
        comm = "torch.distributed"
    elif comm == "auto":
        comm = "xgmi" if world > 1 else "none"

    def build(comm):
        transport = None
        if world > 1:
            if runtime == "native":
                transport = NativeBuffers(layout.plan(rank), phys.F, dtype, device)
            else:
                transport = TorchDistTransport(layout.plan(rank), phys.F, dtype, device)
        eng = Engine(phys, layout, rank, grid=grid, dtype=dtype, device=device, transport=transport,
                     backend=backend, integrator=a.integrator, dt=a.dt)
        runner = None
        if runtime == "persistent":
            from stsphere.ops.persistent import PersistentStepper
            runner = PersistentStepper(eng, timeout_s=5.0, max_steps_per_launch=1000)
        elif runtime == "native":
            # C++ runtime, hipGraph replay; between GPUs either direct xGMI
            # stores from the stage kernels (graph-captured) or RCCL grouped
            # P2P on a high-priority stream + interior/boundary overlap (eager)
            from stsphere.ops.native_runtime import NativeStepper, create_nccl_comm
            xg = None
            nc = None
            if comm == "xgmi":
                from stsphere.ops.xgmi import XgmiHalo
                xg = XgmiHalo(eng, timeout_s=2.0)
            elif comm == "rccl":
                nc = create_nccl_comm(rank, world, local)
            runner = NativeStepper(eng, nccl_comm=nc, use_graph=True, steps_per_graph=a.steps_per_graph, xgmi=xg)
        elif runtime == "graph":
            runner = GraphStepper(eng, a.steps_per_graph)
        return eng, runner

    def agree(ok: bool) -> bool:
        if world == 1:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    try:
        eng, runner = build(comm)
        ok = True
    except Exception as exc:   # e.g. no IPC between these GPUs
        print(f"[bench] rank {rank}: {comm} setup failed: {exc}", file=sys.stderr, flush=True)
        ok = False
    if comm == "xgmi" and not agree(ok):
        comm = "rccl"
        eng, runner = build(comm)
    elif not ok:
        raise SystemExit(1)
    step = runner.run if runner is not None else eng.step

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    step(a.warmup)
    sync()
    if comm == "xgmi":
        ok = True
        try:
            runner.check()
        except RuntimeError as exc:
            print(f"[bench] rank {rank}: {exc}", file=sys.stderr, flush=True)
            ok = False
        if not agree(ok):   # fall back to RCCL from a fresh state
            comm = "rccl"
            eng, runner = build(comm)
            step = runner.run
            step(a.warmup)
            sync()
    t0 = time.perf_counter()
    step(a.steps)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if runtime in ("persistent", "native"):
        runner.check()
    diag = eng.diagnostics()
    if world > 1:
        t = torch.tensor([diag.get("mass", 0.0)], dtype=torch.float64, device=device)
        dist.all_reduce(t)
        diag["mass"] = float(t.item())
    finite = bool(torch.isfinite(eng.tiles_view()).all().item())
    verified = None
    if world > 1 and not a.no_verify:
        # the multi-GPU result must equal a one-GPU run of the same steps bit for
        # bit (same kernels, same arithmetic); rank 0 re-runs it after timing
        tiles = eng.tiles_view().detach().cpu().numpy()
        allt = [None] * world
        dist.all_gather_object(allt, tiles)
        if rank == 0:
            verified = verify_single(a, phys, grid, dtype, device, eng.dt, layout, allt, runtime, backend)
    cells = 6 * a.N * a.N
    cups = cells * a.steps / elapsed
    sdpd = (a.steps * eng.dt / DAY) / (elapsed / DAY)
    if rank == 0:
        out = {
            "metric": "cell-updates/sec (whole node) at C96",
            "value": cups,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * elapsed / a.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": cups / BASELINE_CUPS,
            "dtype": "fp64" if dtype == torch.float64 else "fp32",
            "data": "synthetic (Williamson TC5 analytic initial condition on a random-free C96 grid)",
            "config": {
                "model": f"cubed-sphere shallow water, Williamson {a.case.upper()}, C{a.N}, SSP-RK3 FV-PLR (MC limiter, Rusanov)",
                "global_batch": 1,
                "seq_len": cells,
                "parallelism": f"spatial tiles: {layout.num_tiles} tiles over {world} GPU(s), {layout.partition} partition",
                "N": a.N,
                "tiles_per_edge": a.tiles_per_edge,
                "integrator": a.integrator,
                "dt_s": eng.dt,
                "backend": backend,
                "runtime": runtime,
                "comm": comm,
            },
            "simulated_days_per_day": sdpd,
            "finite": finite,
            "max_abs_diff_vs_1gpu": verified,
            "mass": diag.get("mass"),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
