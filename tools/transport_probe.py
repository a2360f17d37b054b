#!/usr/bin/env python
"""The exchange transports of the stage-kernel runtime, measured in ONE process
on one GPU with the loopback layout (every other tile's ghosts cross the
transport, the rank being its own peer): RCCL grouped send/recv (eager op
list), IPC copies (graph-replayed), direct xGMI rings inside the stage
kernels (graph-replayed), against the same grid without any exchange.  The
loopback path runs the full multi-GPU code path (pack, comm stream, interior
/ boundary split) without a second GPU.  One JSON line.

    python tools/transport_probe.py [--N 96] [--t 2] [--steps 60]
"""
import argparse
import json
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--t", type=int, default=2)
    ap.add_argument("--steps", type=int, default=60)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops import native_runtime as nr
    from stsphere.ops.native_runtime import IpcExchange, NativeStepper
    from stsphere.ops.xgmi import XgmiHalo
    from stsphere.parallel.comm import NativeBuffers
    from stsphere.parallel.layout import TileLayout
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    dev = torch.device("cuda")
    grid = CubedSphereGrid(a.N)
    out = {"N": a.N, "t": a.t, "steps": a.steps}

    def engine(loopback):
        L = TileLayout(a.N, a.t, 1, ng=2, loopback=loopback)
        tr = NativeBuffers(L.plan(0), 4, torch.float64, dev) if loopback else None
        return Engine(ShallowWater("tc5"), L, grid=grid, device=dev, backend="hip", transport=tr)

    def timed(runner, label):
        runner.prepare(a.steps) if hasattr(runner, "prepare") else None
        runner.run(a.steps)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        runner.run(a.steps)
        e1.record()
        torch.cuda.synchronize()
        runner.check()
        out[f"{label}_us_per_step"] = round(e0.elapsed_time(e1) * 1e3 / a.steps, 2)
        st = dict(runner.stats)
        out[f"{label}_graph_steps"] = st.get("graph_steps")
        out[f"{label}_eager_steps"] = st.get("eager_steps")

    e = engine(False)
    r = NativeStepper(e, use_graph=True, steps_per_graph=a.steps)
    timed(r, "no_exchange")
    r.close()
    # direct xGMI rings in the stage kernels
    e = engine(True)
    xg = XgmiHalo(e)
    r = NativeStepper(e, use_graph=True, steps_per_graph=a.steps, xgmi=xg)
    timed(r, "xgmi")
    r.close()
    xg.close()
    # IPC copies, graph-replayed
    e = engine(True)
    ipc = IpcExchange(e, IpcExchange.slots_for(e))
    r = NativeStepper(e, use_graph=True, steps_per_graph=a.steps, ipc=ipc)
    timed(r, "ipc")
    r.close()
    ipc.close()
    # RCCL grouped send/recv, eager op list
    e = engine(True)
    comm = nr.create_nccl_comm(0, 1, 0)
    r = NativeStepper(e, nccl_comm=comm, use_graph=True, steps_per_graph=a.steps)
    timed(r, "rccl")
    r.close()
    nr.lib().stsp_nccl_comm_destroy(comm)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
