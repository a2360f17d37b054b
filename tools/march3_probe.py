#!/usr/bin/env python
"""Time the pieces of the pipelined streaming step (ops/march3.py) on one GPU:
the march launch alone, the two band launches alone, and the whole step, each
as a hipGraph of --reps back-to-back launches (event-timed), plus the
three-launch streaming stage for comparison.  One JSON line.

    python tools/march3_probe.py --N 720 --dtype fp64 --rows 32
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=720)
    ap.add_argument("--t", type=int, default=1)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-stage", action="store_true", help="skip the three-launch streaming-stage row")
    a = ap.parse_args()
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops import native
    from stsphere.ops.march3 import BAND_BLOCK, March3Step
    from stsphere.parallel.layout import TileLayout
    dtype = torch.float64 if a.dtype == "fp64" else torch.float32
    e = Engine(ShallowWater("tc5"), TileLayout(a.N, a.t, 1, ng=2), grid=CubedSphereGrid(a.N), dtype=dtype,
               device="cuda", backend="hip")
    m3 = March3Step(e, rows=a.rows)
    L = native.require_native()
    hc = e.compute
    d, m, band = m3.step_descs(e.pool[0], m3.extra)
    s = torch.cuda.Stream()

    def march(st):
        native.check(L.stsp_march3_launch(hc.dcode, a.rows, ctypes.byref(d), ctypes.byref(m), st), "march3")

    def bands(st):
        for bd in band:
            native.check(L.stsp_stage_launch(hc.phys_id, hc.dcode, BAND_BLOCK[0], BAND_BLOCK[1], ctypes.byref(bd), st),
                         "band")

    def step(st):
        march(st)
        bands(st)

    def stage3(st):
        for stg in e.integ.stages:
            hc.launch(hc.desc(stg, e.dt, None, hc.nblocks), st)

    def timed(fn):
        with torch.cuda.stream(s):
            fn(s.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(a.reps):
                fn(s.cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            g.replay()
            t1.record()
            torch.cuda.synchronize()
            us = 1e3 * t0.elapsed_time(t1) / a.reps
            best = us if best is None else min(best, us)
        return best

    out = {"N": a.N, "t": a.t, "dtype": a.dtype, "rows": a.rows, "band_blocks": int(m3.band.numel()), "D": m3.D,
           "jobs": int(e.plan.T * m3.ncs * m3.nrs)}
    out["march_us"] = timed(march)
    out["band_us"] = timed(bands)
    out["step_us"] = timed(step)
    if not a.no_stage and hc.march:
        out["stage3_us"] = timed(stage3)
    cells = 6 * a.N * a.N
    out["step_cups"] = cells / (out["step_us"] * 1e-6)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
