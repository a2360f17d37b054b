#!/usr/bin/env python
"""Headline benchmark: cell-updates/s (whole node) of the cubed-sphere
shallow-water solver at C96 (BASELINE.json metric), plus simulated-days/day.

Flagship step: Williamson TC5 (zonal flow over a mountain; synthetic initial
condition, nothing downloaded), C96 = 6 x 96^2 cells, float64, SSP-RK3 (every
RK stage of every step is computed by the fused gfx950 stage kernels), 24
tiles of 48^2 (tiles_per_edge = 2) so the same decomposition runs on 1, 2, 4
and 8 GPUs (corner partition: a rank owns the 3 face-quadrants around each
cube vertex it holds).  Strong scaling: the C96 problem is fixed as N grows.

    python bench.py                              # 1 GPU
    python bench.py --gpus 8                     # spawns 8 ranks (torch.distributed.run)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints one JSON line.  Order of events on every rank:

  1. build the engine and the step runner (hipGraph replay of the native op
     list; between GPUs the direct xGMI exchange, RCCL as fallback);
  2. ``prepare(K)``: record the graph(s) ``run(K)`` replays and replay them
     once on a scratch copy of the state (instantiate/upload outside timing);
  3. W warmup steps;
  4. N > 1: the warmup state is compared with a one-GPU run of the same W
     steps (must be bit-identical) BEFORE timing; a mismatch or a poll
     timeout falls back to RCCL from a fresh state, a second mismatch aborts;
  5. barrier + synchronize, exactly K steps, synchronize + barrier; the time
     is the max over ranks; the runner's counters must show K graph-replayed
     steps and no eager ones where a graph path was chosen.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

BASELINE_CUPS = 2.6e8   # derived FV-PLR roofline cell-updates/s (900 GB/s device)


def parse(argv=None):
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
    ap.add_argument("--runtime", default="auto", choices=["auto", "fused", "native", "graph", "eager"],
                    help="fused: one launch per SSP-RK3 step (temporal blocking, one rank); native: one launch "
                         "per RK stage (C++ op list, any rank count); auto: fused where it applies")
    ap.add_argument("--steps-per-launch", type=int, default=0,
                    help="fused runtime: steps inside one kernel launch (0 = auto: the largest even divisor of "
                         "--steps up to 512 when every block fits on the GPU at once; 1 = one launch per step)")
    ap.add_argument("--launch", default="auto", choices=["auto", "direct", "graph"],
                    help="fused runtime: issue each multi-step kernel launch directly or replay it from a "
                         "hipGraph (a one-kernel graph only adds hipGraphLaunch's host floor); auto: direct on "
                         "one GPU, graph across GPUs (the path the multi-rank rehearsals validated)")
    ap.add_argument("--steps-per-graph", type=int, default=0,
                    help="steps recorded per graph (0 = the whole timed run in one graph)")
    ap.add_argument("--comm", default="auto", choices=["auto", "xgmi", "ipc", "rccl"],
                    help="multi-GPU halo exchange of the native runtime: direct xGMI stores from the stage "
                         "kernels (graph-captured; default), IPC copies into the peers' receive slots "
                         "(a copy+signal kernel and a wait kernel, graph-captured) or RCCL grouped send/recv "
                         "(eager)")
    ap.add_argument("--march3", default="auto", choices=["auto", "on", "off"],
                    help="native runtime, one rank, streaming-stage grids: the pipelined SSP-RK3 march (one "
                         "launch per step for the tile interiors + two band launches, ops/march3.py) instead of "
                         "three streaming-stage launches; auto: the measured-faster choice (currently the three "
                         "launches, profiles/r6_march3)")
    ap.add_argument("--march3-rows", type=int, default=0, help="pipelined march: stage-3 rows per wave (0 = auto)")
    ap.add_argument("--partition", default="auto")
    ap.add_argument("--dt", type=float, default=None)
    ap.add_argument("--block", default=None, help="stage block shape BXxBY, or the fused runtime's square block size B (default: chosen per grid)")
    ap.add_argument("--timeout", type=float, default=float(os.environ.get("STSP_BENCH_TIMEOUT", "480")),
                    help="--gpus N > 1 (self-launched): kill every rank and print a status=timeout JSON line "
                         "after this many seconds (0 = no deadline)")
    ap.add_argument("--sync", default="spin", choices=["spin", "auto"],
                    help="host wait mode of the GPU: spin (hipDeviceScheduleSpin) or the runtime default")
    ap.add_argument("--repeat", type=int, default=0,
                    help="diagnostics: time R more regions of --steps steps after the measured one "
                         "(reported as repeat_ms_per_step; the state then has advanced further)")
    ap.add_argument("--no-verify", action="store_true",
                    help="N > 1: skip the bitwise comparisons with a one-GPU run")
    return ap.parse_args(argv)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _phase(name: str) -> None:
    """Record this rank's current phase (read by the launching parent when the
    run overruns its deadline)."""
    d = os.environ.get("STSP_PHASE_DIR")
    if d:
        try:
            with open(os.path.join(d, f"rank{os.environ.get('RANK', '0')}.phase"), "w") as f:
                f.write(f"{name} {time.time():.3f}\n")
        except OSError:
            pass


def _fail_line(a, status: str, **extra) -> str:
    """The one JSON line of a run that produced no measurement."""
    out = {"metric": f"cell-updates/sec (whole node) at C{a.N}", "value": None, "unit": "cell-updates/s",
           "n_gpus": a.gpus, "steps": a.steps, "warmup": a.warmup, "ms_per_step": None,
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": a.dtype,
           "data": "synthetic", "status": status}
    out.update(extra)
    return json.dumps(out)


def launch_ranks(a) -> int:
    """--gpus N > 1 without a distributed launch: start N fresh worker
    processes with torch.distributed.run (this parent never touches the GPU,
    and is never replaced by exec) and pass their output through; rank 0 prints
    the JSON line.  Returns the launcher's exit code.

    Deadline: the workers run in their own process group; past ``--timeout``
    seconds the whole group is killed and this parent prints one JSON line with
    ``"status": "timeout"`` and the last phase each rank reached (each rank
    writes its phase to a file in a scratch directory), then exits non-zero."""
    import shutil
    import signal
    import tempfile
    share = os.environ.get("STSP_SHARE_GPU") == "1"
    if a.backend == "hip" and not share:
        import torch   # device_count() does not initialise the GPU
        have = torch.cuda.device_count()
        if have < a.gpus:
            print(_fail_line(a, "error", error=f"--gpus {a.gpus} but only {have} GPU(s) visible "
                                               "(STSP_SHARE_GPU=1 rehearses several ranks on one GPU)"),
                  flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if share and a.comm != "ipc" and os.environ.get("STSP_FAIL_XGMI") != "1":
        # several ranks on ONE GPU: one hardware queue per process.  With the
        # default four, three or more processes oversubscribe the queues the
        # scheduler maps at once, it time-slices them, and a multi-step fused
        # kernel (every rank's blocks resident together) times out
        # (profiles/r5_rehearse/README.md).  A real node has a GPU per rank.
        # (The box exports GPU_MAX_HW_QUEUES=4, so this overrides it;
        # STSP_SHARE_HW_QUEUES chooses another count.  Not for the IPC copy
        # transport: its comm-stream copies and graph replays crashed inside
        # hipGraphLaunch with one queue per process, and it needs no
        # co-residency, only its bounded spin-wait kernels.)
        env["GPU_MAX_HW_QUEUES"] = os.environ.get("STSP_SHARE_HW_QUEUES", "1")
    env.setdefault("OMP_NUM_THREADS", "1")
    pdir = tempfile.mkdtemp(prefix="stsp_phase_")
    env["STSP_PHASE_DIR"] = pdir
    t0 = time.time()
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return proc.wait(timeout=a.timeout if a.timeout > 0 else None)
    except subprocess.TimeoutExpired:
        phases = {}
        for r in range(a.gpus):
            try:
                with open(os.path.join(pdir, f"rank{r}.phase")) as f:
                    name, ts = f.read().split()
                phases[str(r)] = {"phase": name, "since_s": round(time.time() - float(ts), 1)}
            except (OSError, ValueError):
                phases[str(r)] = {"phase": "not started", "since_s": None}
        for sig, grace in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                break
            try:
                proc.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        print(_fail_line(a, "timeout", timeout_s=a.timeout, elapsed_s=round(time.time() - t0, 1), phases=phases),
              flush=True)
        return 124
    finally:
        shutil.rmtree(pdir, ignore_errors=True)


def single_rank_reference(a, phys_factory, grid, dtype, device, dt, ng, nsteps, runtime, backend, fused_B=None):
    """[F, 6, N, N] state of one rank stepping ``nsteps`` from the initial
    condition on this device (the bitwise reference of a multi-rank run).
    ``fused_B``: the ranks' fused block size (the panel-edge normals and lengths
    of a face come from in-kernel tangents inside one panel and from host
    tables in edge blocks, so the block size moves results by roundoff)."""
    import numpy as np
    from stsphere.engine import Engine
    from stsphere.parallel.layout import TileLayout
    L1 = TileLayout(a.N, a.tiles_per_edge, 1, ng=ng)
    ref = Engine(phys_factory(), L1, 0, grid=grid, dtype=dtype, device=device, backend=backend,
                 integrator=a.integrator, dt=dt)
    if runtime in ("native", "fused") and backend == "hip":
        from stsphere.ops.native_runtime import NativeStepper
        fk = None
        if runtime == "fused":
            from stsphere.ops.fused import FusedKernel
            fk = FusedKernel(ref, B=fused_B)
        r = NativeStepper(ref, use_graph=True, steps_per_graph=max(nsteps, 1), fused=fk)
        r.run(nsteps)
        r.close()
    else:
        ref.step(nsteps)
    return np.stack([ref.global_field(f) for f in range(ref.physics.F)])


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    import numpy as np
    import torch
    import torch.distributed as dist
    from stsphere.engine import Engine, GraphStepper, assemble_global
    from stsphere.models.geometry import CubedSphereGrid, DAY
    from stsphere.models.swe import ShallowWater
    from stsphere.parallel.comm import NativeBuffers, TorchDistTransport
    from stsphere.parallel.layout import TileLayout

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # STSP_SHARE_GPU=1: rehearsal mode, every rank on cuda:0 with a gloo group
    # (functional check of the multi-rank paths on a one-GPU box; not a benchmark)
    share = os.environ.get("STSP_SHARE_GPU") == "1"
    cpu = a.backend == "torch" and os.environ.get("STSP_BENCH_DEVICE", "") == "cpu"
    # host waits spin (set before torch creates the device context): the timed
    # region ends with a synchronize, and a blocking wait adds its wake-up
    spin_rc = None
    if a.sync == "spin" and not cpu and a.backend == "hip" and torch.cuda.device_count() > 0:
        from stsphere.ops import native as _native
        spin_rc = int(_native.load(build_if_missing=False).stsp_schedule_spin(0 if share else local))
    use_gpu = (not cpu) and torch.cuda.is_available()
    device = torch.device(f"cuda:{0 if share else local}") if use_gpu else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1:
        _phase("init_process_group")
        if device.type == "cuda" and not share:
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    dtype = torch.float64 if a.dtype == "fp64" else torch.float32
    ng = 2
    layout = TileLayout(a.N, a.tiles_per_edge, world, ng=ng, partition=a.partition)
    grid = CubedSphereGrid(a.N)
    phys_factory = lambda: ShallowWater(a.case)
    phys = phys_factory()
    backend = a.backend if device.type == "cuda" else "torch"
    runtime = a.runtime
    if runtime == "auto":
        runtime = "native" if (device.type == "cuda" and backend == "hip") else "eager"
        if runtime == "native" and (world == 1 or a.comm in ("auto", "xgmi")):
            from stsphere.ops.fused import fused_block, fused_supported_config, rank_cus
            # the fused step recomputes a ring of 2 x 3 cells per block: it wins
            # where launches and hand-offs dominate (every block resident, so
            # several steps run per launch); larger grids keep the stage path.
            # One GPU up to two passes over the CUs: one fused launch per step still
            # beats three stage launches (C180, 3 tiles per edge, 486 blocks: 38.6 vs
            # 44.5 us/step, profiles/r3_march/c180_fused_b20.log)
            cus = rank_cus(device) if device.type == "cuda" else 256
            ntl = len(layout.rank_tiles[rank])
            B = fused_block(layout.n, ntl, cus)
            nb = ntl * (layout.n // B) ** 2 if B else None
            if nb is not None and (nb <= cus or (world == 1 and nb <= 2 * cus)) and \
                    fused_supported_config(phys, a.integrator, layout, B) is None:
                runtime = "fused"
    comm = a.comm if world > 1 else "none"
    if world > 1 and runtime == "fused":
        comm = "xgmi"                    # remote window cells through the fused kernel's xGMI ring
    elif world > 1 and runtime not in ("native", "fused"):
        comm = "torch.distributed"
    elif comm == "auto":
        comm = "xgmi" if world > 1 else "none"
    spg = a.steps_per_graph if a.steps_per_graph > 0 else a.steps
    info = {"steps_per_launch": None}

    # collectives on CUDA tensors with RCCL, on CPU tensors with gloo
    cdev = device if (world > 1 and dist.get_backend() == "nccl") else torch.device("cpu")

    def agree(ok: bool) -> bool:
        if world == 1:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
            if device.type == "cuda":
                torch.cuda.synchronize(device)

    # bound of every in-kernel wait for another rank (the kernels set an error
    # word instead of hanging).  Ranks sharing one GPU (rehearsals) can be
    # time-sliced by the scheduler for longer than a real node ever waits
    # (six processes: profiles/r5_rehearse/README.md), hence the longer bound
    xg_timeout = float(os.environ.get("STSP_XG_TIMEOUT", "30" if share else "2"))

    def build(comm):
        transport = None
        if world > 1:
            if runtime in ("native", "fused"):
                transport = NativeBuffers(layout.plan(rank), phys.F, dtype, device)
            else:
                transport = TorchDistTransport(layout.plan(rank), phys.F, dtype, device)
        blk = tuple(int(v) for v in a.block.lower().split("x")) if a.block and "x" in a.block.lower() else None
        eng = Engine(phys_factory(), layout, rank, grid=grid, dtype=dtype, device=device, transport=transport,
                     backend=backend, integrator=a.integrator, dt=a.dt, block=blk)
        runner, xg = None, None
        if runtime == "fused":
            # one launch per SSP-RK3 step (temporal blocking, ops/fused.py), hipGraph replay;
            # between GPUs the remote window cells travel through the kernel's own xGMI ring
            from stsphere.ops.fused import FusedKernel, rank_cus as _rank_cus
            from stsphere.ops.native_runtime import NativeStepper
            fB = int(a.block) if a.block and a.block.isdigit() else None    # --block B: the fused block size
            fk = FusedKernel(eng, B=fB, timeout_s=xg_timeout)      # collective with several ranks
            xg = fk if world > 1 else None
            spl = a.steps_per_launch
            if spl == 0:
                # several steps per launch (in-kernel producer waits) need every block resident;
                # the longest even launch that divides the timed steps (each launch boundary
                # costs ~18 us of ramp: 300 steps in one launch 12.05 us/step against 12.09-12.18
                # in 60-step launches, profiles/r4_spl/)
                cus = _rank_cus(device)
                spl = max([k for k in range(2, 513, 2) if a.steps % k == 0], default=1) if fk.plan.nb <= cus else 1
            info["steps_per_launch"] = spl
            info["fused_B"] = fk.plan.B
            runner = NativeStepper(eng, use_graph=True, steps_per_graph=spg, fused=fk, steps_per_launch=spl,
                                   direct=a.launch == "direct" or (a.launch == "auto" and world == 1))
        elif runtime == "native":
            # C++ runtime, hipGraph replay; between GPUs either direct xGMI
            # stores from the stage kernels (graph-captured) or RCCL grouped
            # P2P on a high-priority stream + interior/boundary overlap (eager)
            from stsphere.ops.native_runtime import IpcExchange, NativeStepper, create_nccl_comm
            nc = ipc = None
            if comm == "xgmi":
                from stsphere.ops.xgmi import XgmiHalo
                xg = XgmiHalo(eng, timeout_s=xg_timeout)      # collective; raises on every rank alike
            elif comm == "ipc":
                ipc = xg = IpcExchange(eng, IpcExchange.slots_for(eng), timeout_s=xg_timeout)   # collective
            elif comm == "rccl":
                nc = create_nccl_comm(rank, world, local)
            m3 = None
            if world == 1 and a.march3 != "off":
                from stsphere.ops.march3 import March3Step, march3_unsupported, march3_wanted
                if a.march3 == "on" or march3_wanted(eng):
                    why = march3_unsupported(eng)
                    if why:
                        raise SystemExit(f"[bench] --march3 on: {why}")
                    m3 = March3Step(eng, rows=a.march3_rows or 32)
                    info["march3_rows"] = m3.rows
            runner = NativeStepper(eng, nccl_comm=nc, use_graph=True, steps_per_graph=spg,
                                   xgmi=xg if comm == "xgmi" else None, ipc=ipc, march3=m3)
        elif runtime == "graph":
            runner = GraphStepper(eng, spg)
        return eng, runner, xg

    def close(runner, xg):
        for obj in (runner, xg):
            if obj is not None and hasattr(obj, "close"):
                try:
                    obj.close()
                except Exception as exc:   # best effort; the fresh build follows
                    print(f"[bench] rank {rank}: close failed: {exc}", file=sys.stderr, flush=True)

    def warm(eng, runner):
        """prepare(K) + W warmup steps; False if the exchange timed out."""
        if hasattr(runner, "prepare"):
            runner.prepare(a.steps)
        step = runner.run if runner is not None else eng.step
        step(a.warmup)
        sync()
        # one rank: the exchange check is the post-timing one (runner.check() below);
        # a device read here only lengthens the GPU's idle gap before the timed region.
        # (Round 6 also tried skipping this sync so the host work before the timed
        # region overlaps the last warm-up launches: the GPU idled 26 instead of 53 us
        # before the timed launch and the 20-step bench did not change, 13.17-13.60 vs
        # 13.11-13.36 us/step; profiles/r6_handoff/warm_gap.)
        if hasattr(runner, "check") and world > 1:
            try:
                runner.check()
            except RuntimeError as exc:
                print(f"[bench] rank {rank}: {exc}", file=sys.stderr, flush=True)
                return False
        return True

    def gathered(eng):
        tiles = eng.tiles_view().detach().cpu().numpy()
        allt = [None] * world
        dist.all_gather_object(allt, tiles)
        return np.stack([assemble_global(layout, {r: t[f] for r, t in enumerate(allt)}) for f in range(phys.F)])

    def diff_vs_1gpu(eng, nsteps):
        """max |multi-rank - one rank| after nsteps (0.0 = bitwise), on every rank."""
        got = gathered(eng)
        d = torch.zeros(1, dtype=torch.float64, device=cdev)
        if rank == 0:
            want = single_rank_reference(a, phys_factory, grid, dtype, device, eng.dt, ng, nsteps, runtime, backend,
                                         fused_B=info.get("fused_B") if runtime == "fused" else None)
            d[0] = float(np.abs(got - want).max())
        dist.broadcast(d, src=0)
        return float(d.item())

    # transport fallback chain between GPUs: the direct xGMI rings, then the
    # graph-captured IPC copy transport, then eager RCCL; each attempt is
    # agreed by every rank (setup, warmup exchange check, bitwise check
    # against one GPU) and a failed one restarts from a fresh state
    FALLBACK = {"xgmi": "ipc", "ipc": "rccl"}
    chain = [comm]
    while world > 1 and chain[-1] in FALLBACK:
        chain.append(FALLBACK[chain[-1]])
    eng = runner = xg = None
    fallback_reason = None
    warm_diff = None
    verify = world > 1 and not a.no_verify

    def attempt(c):
        """(engine, runner, exchange, ok, why) of one transport."""
        e_ = r_ = x_ = None
        why = None
        _phase(f"build_{c}")
        try:
            e_, r_, x_ = build(c)
            ok_ = True
        except Exception as exc:   # e.g. no IPC between these GPUs
            print(f"[bench] rank {rank}: {c} setup failed: {exc}", file=sys.stderr, flush=True)
            why = f"rank {rank}: {c} setup failed: {exc}"
            ok_ = False
        if world > 1 and not agree(ok_):
            return e_, r_, x_, False, why or f"{c} setup failed on another rank", None
        if not ok_:
            raise SystemExit(1)
        _phase(f"warmup_{c}")
        if os.environ.get("STSP_BENCH_HANG_RANK") == str(rank):   # test hook: a rank that never returns
            while True:
                time.sleep(1)
        ok_ = warm(e_, r_)
        if not ok_:
            why = f"rank {rank}: {c} exchange timed out in warmup"
        d_ = None
        if verify and ok_:
            _phase(f"verify_{c}")
            d_ = diff_vs_1gpu(e_, a.warmup)
            ok_ = d_ == 0.0
            if not ok_:
                why = f"{c}: warmup state differs from one GPU by {d_:.3e}"
                if rank == 0:
                    print(f"[bench] {why}", file=sys.stderr, flush=True)
        if world > 1 and not agree(ok_):
            return e_, r_, x_, False, why or f"{c} check failed on another rank", d_
        return e_, r_, x_, True, None, d_

    for k, c in enumerate(chain):
        if k:
            runtime = "native" if runtime == "fused" else runtime   # the fallbacks are stage-kernel op lists
        eng, runner, xg, ok, why, warm_diff = attempt(c)
        if ok:
            comm = c
            break
        fallback_reason = why if fallback_reason is None else f"{fallback_reason}; {why}"
        close(runner, xg)
        if k == len(chain) - 1:
            raise SystemExit(f"[bench] rank {rank}: every transport failed ({fallback_reason})")
    _phase("timed_prep")
    step = runner.run if runner is not None else eng.step
    stats0 = dict(getattr(runner, "stats", {}))
    _phase("timed")
    sync()
    t0 = time.perf_counter()
    step(a.steps)
    sync()
    elapsed = time.perf_counter() - t0
    stats1 = dict(getattr(runner, "stats", {}))
    timed = {k: stats1[k] - stats0.get(k, 0) for k in stats1}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # diagnostics only (--repeat R): R more timed regions of the same K steps
    # after the measured one, reported separately (the headline is the first)
    repeats = []
    for _ in range(a.repeat):
        sync()
        t1 = time.perf_counter()
        step(a.steps)
        sync()
        repeats.append(1e3 * (time.perf_counter() - t1) / a.steps)
    if hasattr(runner, "check"):
        runner.check()
    graph_path = runtime in ("native", "fused") and getattr(runner, "use_graph", False) \
        and not getattr(runner, "_cxx_graph", False)
    if graph_path and (timed.get("eager_steps", 0) != 0 or timed.get("graph_steps", 0) != a.steps):
        raise SystemExit(f"[bench] timed region was not a pure graph replay: {timed}")
    if getattr(runner, "direct", False) and (timed.get("eager_steps", 0) != 0 or timed.get("direct_steps", 0) != a.steps):
        raise SystemExit(f"[bench] timed region was not whole direct fused launches: {timed}")
    diag = eng.diagnostics()
    if world > 1:
        t = torch.tensor([diag.get("mass", 0.0)], dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        diag["mass"] = float(t.item())
    finite = bool(torch.isfinite(eng.tiles_view()).all().item())
    _phase("final_verify")
    final_diff = diff_vs_1gpu(eng, a.warmup + a.steps) if verify else None
    cells = 6 * a.N * a.N
    cups = cells * a.steps / elapsed
    sdpd = (a.steps * eng.dt / DAY) / (elapsed / DAY)
    if rank == 0:
        out = {
            "metric": f"cell-updates/sec (whole node) at C{a.N}",
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
            "data": f"synthetic (Williamson {a.case.upper()} analytic initial condition on the C{a.N} grid, "
                    "random-free)",
            "config": {
                "model": f"cubed-sphere shallow water, Williamson {a.case.upper()}, C{a.N}, "
                         f"{a.integrator.upper()} FV-PLR (MC limiter, Rusanov)",
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
                "block": list((eng.compute.bx, eng.compute.by)) if hasattr(eng.compute, "bx") else None,
                "steps_per_launch": info["steps_per_launch"],
                "fused_block": info.get("fused_B"),
                "march3_rows": info.get("march3_rows"),
                "graph_replayed_steps": timed.get("graph_steps"),
                "direct_launch_steps": timed.get("direct_steps"),
                "kernel_launches": timed.get("launches") if timed.get("direct_steps") else None,
                "eager_steps": timed.get("eager_steps"),
                "host_sync": a.sync if spin_rc is not None else "auto",
                "host_sync_rc": spin_rc,
            },
            "simulated_days_per_day": sdpd,
            "finite": finite,
            "max_abs_diff_vs_1gpu_warmup": warm_diff,
            "max_abs_diff_vs_1gpu": final_diff,
            "comm_fallback_reason": fallback_reason,
            "status": "ok",
            "mass": diag.get("mass"),
        }
        if repeats:
            out["repeat_ms_per_step"] = repeats
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
