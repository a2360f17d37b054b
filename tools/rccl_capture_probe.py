#!/usr/bin/env python
"""RCCL under hipGraph capture, on one GPU: the loopback layout routes every
ghost of a C24 (or --N) shallow-water step through pack -> grouped RCCL
send/recv to self -> receive-buffer gather, i.e. the complete multi-GPU RCCL
op list.  With STSP_GRAPH_COMM=1 the op list is recorded into a graph (round 3:
RCCL 2.26.6, torch's copy, crashed there).  Run one configuration per process
(a crash ends the process); the RCCL environment (NCCL_GRAPH_MIXING_SUPPORT,
NCCL_GRAPH_REGISTER, ...) is whatever the caller exports.  One JSON line:
bitwise equality with the single-rank engine, graph replay counts, and eager /
replayed us per step.

    STSP_GRAPH_COMM=1 NCCL_GRAPH_MIXING_SUPPORT=0 python tools/rccl_capture_probe.py
    STSP_RCCL_LIB=/opt/rocm/lib/librccl.so.1.0.70200 STSP_GRAPH_COMM=1 python tools/rccl_capture_probe.py

(STSP_RCCL_LIB: ROCm 7.2's RCCL 2.27.7 beside torch's 2.26.6, ops/csrc/runtime.cpp.)
"""
import argparse
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=24)
    ap.add_argument("--steps", type=int, default=60)
    a = ap.parse_args()
    import faulthandler
    faulthandler.enable()        # a crash inside capture / replay names its Python frame
    import torch
    import torch.distributed as dist
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops import native_runtime as nr
    from stsphere.parallel.comm import NativeBuffers
    from stsphere.parallel.layout import TileLayout

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    comm = nr.create_nccl_comm(0, 1, 0)
    out = {"rccl_version": nr.rccl_version() if hasattr(nr, "rccl_version") else None,
           "rccl_path": nr.lib().stsp_rccl_path().decode(),
           "env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "STSP_GRAPH"))}}
    g = CubedSphereGrid(a.N)
    ref = Engine(ShallowWater("tc5"), TileLayout(a.N, 2, 1, ng=2), grid=g, device="cuda", backend="hip")
    L = TileLayout(a.N, 2, 1, ng=2, loopback=True)
    p = L.plan(0)

    def make():
        e = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", dt=ref.dt,
                   transport=NativeBuffers(p, 4, torch.float64, torch.device("cuda")))
        return e

    e = make()
    ns = nr.NativeStepper(e, nccl_comm=comm, use_graph=True, steps_per_graph=3)
    out["graph_capture_enabled"] = bool(ns.use_graph)
    print(f"[probe] {out['rccl_path']} v{out['rccl_version']}: stepper built, running 6 steps", file=sys.stderr,
          flush=True)
    ref.step(6)
    ns.run(6)
    torch.cuda.synchronize()
    out["bitwise_equal_6"] = bool(torch.equal(ref.tiles_view(), e.tiles_view()))
    out["stats_6"] = dict(ns.stats)
    # timing: replayed (or eager) op lists, then the eager op list for comparison
    ns.prepare(a.steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ns.run(a.steps)
    torch.cuda.synchronize()
    out["us_per_step"] = (time.perf_counter() - t0) * 1e6 / a.steps
    out["stats"] = dict(ns.stats)
    ref.step(a.steps)
    torch.cuda.synchronize()
    out["bitwise_equal_total"] = bool(torch.equal(ref.tiles_view(), e.tiles_view()))
    ns.close()
    os.environ["STSP_GRAPH_COMM"] = "0"
    e2 = make()
    ns2 = nr.NativeStepper(e2, nccl_comm=comm, use_graph=True, steps_per_graph=3)
    ns2.run(6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ns2.run(a.steps)
    torch.cuda.synchronize()
    out["eager_us_per_step"] = (time.perf_counter() - t0) * 1e6 / a.steps
    ns2.close()
    nr.lib().stsp_nccl_comm_destroy(comm)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
