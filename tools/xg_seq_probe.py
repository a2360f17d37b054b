#!/usr/bin/env python
"""Which step of the multi-rank fused bench sequence times out (shared-GPU
rehearsal, STSP_SHARE_GPU=1)?  Each rank of a C96 layout builds the fused
kernel with its xGMI ring and a graph-replay NativeStepper with K-step
launches, then runs bench.py's warmup sequence one piece at a time, reading
the kernel's error word after each piece:

  warm     the eager period before the first capture (+ restore/prime)
  capture  two graph copies of one period (host only)
  replay0  graph copy 0 on a scratch copy of the state
  replay1  graph copy 1
  restore  state back + prime (collective)
  run5     run(5): a single-step launch and a 4-step launch (eager)
  runK     run(K): one graph replay

One JSON line per rank: per piece the host seconds since a common barrier at
its start and end and the error word after it.  Launched like bench.py:

  STSP_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 \\
      --master-addr 127.0.0.1 --master-port 29533 tools/xg_seq_probe.py --t 2 --K 20
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--t", type=int, default=2)
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--launch", default="graph", choices=["graph", "direct"])
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops import native
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.parallel.comm import NativeBuffers
    from stsphere.parallel.layout import TileLayout
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    native.load(build_if_missing=False).stsp_schedule_spin(0)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    L = TileLayout(a.N, a.t, world, ng=2)
    phys = ShallowWater("tc5")
    eng = Engine(phys, L, rank, grid=CubedSphereGrid(a.N), dtype=torch.float64, device=dev,
                 transport=NativeBuffers(L.plan(rank), phys.F, torch.float64, dev), backend="hip")
    fk = FusedKernel(eng, timeout_s=2.0)
    r = NativeStepper(eng, use_graph=True, steps_per_graph=a.K, fused=fk, steps_per_launch=a.K,
                      direct=a.launch == "direct")
    out = {"rank": rank, "world": world, "t": a.t, "K": a.K, "B": fk.plan.B, "blocks": fk.plan.nb,
           "launch": a.launch, "pieces": []}
    dist.barrier()
    T0 = time.time()

    def piece(name, fn):
        t1 = time.time() - T0
        fn()
        torch.cuda.synchronize(dev)
        t2 = time.time() - T0
        err = [int(x) for x in fk.tens["err"].cpu().tolist()]
        rec = {"name": name, "t0": round(t1, 4), "t1": round(t2, 4), "err": err}
        if err[0]:
            # where progress stopped: per-block completed-step counters
            ep = fk.tens["epoch"].cpu().numpy()
            lo = int(ep.min())
            stuck = [int(b) for b in np.nonzero(ep == lo)[0]]
            org = fk.plan.org
            rec["epoch_min"], rec["epoch_max"] = lo, int(ep.max())
            rec["epoch_hist"] = {str(int(v)): int((ep == v).sum()) for v in np.unique(ep)}
            rec["stuck_blocks"] = [[b, int(org[b, 0]), int(org[b, 1]), int(org[b, 2])] for b in stuck[:24]]
            rec["tiles"] = [int(x) for x in eng.plan.tiles]
        out["pieces"].append(rec)
        return err[0] == 0

    saved = {}
    if a.launch == "graph":
        seq = [("warm", r._warm),
               ("capture", lambda: (r._graph(1, 0), r._graph(1, 1))),
               ("replay0", lambda: (saved.setdefault("s", r._save()), r._graphs[(1, 0)].replay())),
               ("replay1", lambda: r._graphs[(1, 1)].replay()),
               ("restore", lambda: r._restore(saved["s"])),
               ("run5", lambda: r.run(5)),
               ("runK", lambda: r.run(a.K))]
    else:
        seq = [("prepare", lambda: r.prepare(a.K)), ("run5", lambda: r.run(5)), ("runK", lambda: r.run(a.K))]
    for name, fn in seq:
        ok = torch.tensor([1 if piece(name, fn) else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)     # every rank stops after the same piece
        if not int(ok.item()):
            break
    print(json.dumps(out), flush=True)
    dist.barrier()


if __name__ == "__main__":
    main()
