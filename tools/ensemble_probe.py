#!/usr/bin/env python
"""Ensemble concurrency probe (GPU): M members of the C96 TC5 run
(``stsphere.Ensemble``: one native runner, graph and stream per member)
stepped concurrently, against one member.  Reports the aggregate
member-cell-updates/s and checks every member bitwise against the same member
run alone.

    python tools/ensemble_probe.py [--members 1,2,3,4] [--steps 300] [--N 96]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--members", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--tpe", type=int, default=2)
    ap.add_argument("--spg", type=int, default=0, help="steps per graph (0: the whole timed run)")
    a = ap.parse_args()
    import torch
    from stsphere.ensemble import Ensemble
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.engine import Engine
    from stsphere.parallel.layout import TileLayout

    grid = CubedSphereGrid(a.N)
    L = TileLayout(a.N, a.tpe, 1, ng=2)
    spg = a.spg or a.steps
    cells = 6 * a.N * a.N
    res = {"N": a.N, "steps": a.steps, "tiles_per_edge": a.tpe, "steps_per_graph": spg, "dtype": "fp64",
           "model": "SWE TC5, SSPRK3, MC-PLR"}
    for M in [int(m) for m in a.members.split(",")]:
        ens = Ensemble(lambda: ShallowWater("tc5"), L, M, amplitude=1e-4, grid=grid, device="cuda",
                       backend="hip", steps_per_graph=spg)
        init = [e.tiles_view().clone() for e in ens.engines]
        ens.prepare(a.steps)
        ens.prepare(a.warmup)
        ens.run(a.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ens.run(a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        finals = ens.states().clone()
        diffs = []
        for m in range(M):
            e = Engine(ShallowWater("tc5"), L, grid=grid, device="cuda", backend="hip", dt=ens.dt)
            e.set_state(init[m])
            r = NativeStepper(e, use_graph=True, steps_per_graph=a.steps)
            r.run(a.warmup)
            r.run(a.steps)
            torch.cuda.synchronize()
            diffs.append(float((e.tiles_view() - finals[m]).abs().max()))
            r.close()
        ens.close()
        res[M] = {"wall_s": dt, "us_per_member_step": 1e6 * dt / a.steps,
                  "aggregate_cell_updates_per_s": M * cells * a.steps / dt, "max_abs_diff_vs_alone": max(diffs)}
        print(M, json.dumps(res[M]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
