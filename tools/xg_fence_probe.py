#!/usr/bin/env python
"""Cost of the direct-xGMI publish protocol on one GPU (loopback).

A loopback rank sends every ghost through its own receive ring, so each
stage pays the ring stores, the publish fences/atomics and the polls of the
multi-GPU path.  Run once per library variant (STSP_VARIANT = "" | xgf1 |
xgf2, see ops/build.py) and compare µs/step with the plain single-GPU step;
the loopback result must stay bitwise equal to the plain one.

    STSP_VARIANT=xgf2 python tools/xg_fence_probe.py --N 96 --t 2
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
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--block", default=None)
    a = ap.parse_args()
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.ops.xgmi import XgmiHalo
    from stsphere.parallel.comm import NativeBuffers
    from stsphere.parallel.layout import TileLayout
    block = tuple(int(v) for v in a.block.split("x")) if a.block else None
    g = CubedSphereGrid(a.N)
    plain = Engine(ShallowWater("tc5"), TileLayout(a.N, a.t, 1, ng=2), grid=g, device="cuda", backend="hip",
                   block=block)
    L = TileLayout(a.N, a.t, 1, ng=2, loopback=True)
    lb = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", dt=plain.dt, block=block,
                transport=NativeBuffers(L.plan(0), 4, torch.float64, torch.device("cuda")))
    xg = XgmiHalo(lb, timeout_s=1.0)
    rp = NativeStepper(plain, use_graph=True, steps_per_graph=30)
    rx = NativeStepper(lb, use_graph=True, steps_per_graph=30, xgmi=xg)
    out = {"variant": os.environ.get("STSP_VARIANT", ""), "N": a.N, "t": a.t, "block": [lb.compute.bx, lb.compute.by]}
    for name, r in (("plain", rp), ("loopback_xg", rx)):
        r.run(30)
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            r.run(a.steps)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e6
            best = dt if best is None else min(best, dt)
        out[name + "_us_per_step"] = best
    rx.check()
    out["bitwise_equal"] = bool(torch.equal(plain.tiles_view(), lb.tiles_view()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
