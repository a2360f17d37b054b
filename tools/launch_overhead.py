#!/usr/bin/env python
"""Host-side cost of one timed region of the headline bench (C96, 20 fused
steps in one launch), split by layer: the bench's runner.run(20), the fused
kernel's launch(), the bare ctypes launch, and the surrounding synchronise.
Each number is the median over R repetitions of the host time of that call
alone (the GPU work is synchronised away between repetitions), plus the full
region (launch + synchronise) as the bench times it.  One JSON line.

    python tools/launch_overhead.py [--reps 50]
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from stsphere.ops import native
    native.load(build_if_missing=False).stsp_schedule_spin(0)
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.parallel.layout import TileLayout
    L = TileLayout(96, 2, 1, ng=2)
    e = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(96), device="cuda", backend="hip")
    fk = FusedKernel(e)
    r = NativeStepper(e, use_graph=True, steps_per_graph=a.steps, fused=fk, steps_per_launch=a.steps, direct=True)
    r.prepare(a.steps)
    r.run(a.steps)
    torch.cuda.synchronize()
    sync = torch.cuda.synchronize
    out = {"steps": a.steps}

    def med(fn):
        ts = []
        for _ in range(a.reps):
            sync()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        sync()
        return 1e6 * statistics.median(ts)

    out["runner_run_us"] = med(lambda: r.run(a.steps))
    out["fused_launch_us"] = med(lambda: fk.launch(0, nsteps=a.steps))
    d = fk.multi_desc(a.steps)
    st = int(torch.cuda.current_stream().cuda_stream)
    fn = fk._launch_fn
    out["ctypes_launch_us"] = med(lambda: fn(fk.dcode, d, st))
    out["current_stream_us"] = med(lambda: int(torch.cuda.current_stream().cuda_stream))
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        out["raw_stream_us"] = med(lambda: int(raw(0)))
        out["raw_stream_equals"] = int(raw(0)) == st
    out["sync_idle_us"] = med(sync)

    def region():
        t0 = time.perf_counter()
        r.run(a.steps)
        sync()
        return time.perf_counter() - t0
    ts = []
    for _ in range(a.reps):
        sync()
        ts.append(region())
    out["region_us_per_step"] = 1e6 * statistics.median(ts) / a.steps
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gs = []
    for _ in range(10):
        sync()
        e0.record()
        r.run(a.steps)
        e1.record()
        sync()
        gs.append(e0.elapsed_time(e1) * 1e3 / a.steps)
    out["region_gpu_events_us_per_step"] = statistics.median(gs)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
