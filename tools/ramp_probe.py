#!/usr/bin/env python
"""Where the first steps of a multi-step fused launch lose time (C96, the
bench's 20-step region runs ~0.5 µs/step slower than a 100-step launch).

GPU-event time of ONE direct launch of n steps, for a range of n, in two
conditions:
  cold: the GPU idles (host sleep) before the launch, as before bench.py's
        timed region;
  hot:  a ~2 ms busy kernel runs just before the launch on the same stream
        (events bracket the fused launch only), so clocks and power state
        are those of a busy GPU.
The per-step increments T(n) - T(n') separate a one-off prologue (a constant
offset) from a gradual settling of the block pipeline (larger increments at
small n) and from clock ramp (cold slower than hot).  One JSON line.

    python tools/ramp_probe.py [--reps 15]
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
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.fused import FusedKernel
    from stsphere.parallel.layout import TileLayout
    L = TileLayout(96, 2, 1, ng=2)
    e = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(96), device="cuda", backend="hip")
    fk = FusedKernel(e)
    ns = (2, 4, 6, 8, 10, 12, 16, 20, 30, 40, 60, 100)
    for n in ns:
        fk.multi_desc(n)
    fk.launch(0, nsteps=4)
    torch.cuda.synchronize()
    busy_a = torch.randn(2048, 2048, dtype=torch.float64, device="cuda")
    busy_b = torch.empty_like(busy_a)

    def busy():
        for _ in range(8):
            torch.matmul(busy_a, busy_a, out=busy_b)

    def one(n, hot):
        torch.cuda.synchronize()
        if hot:
            busy()
        else:
            time.sleep(0.002)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fk.launch(0, nsteps=n)          # n even: the state ends in pool[0] again
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    out = {"blocks": fk.plan.nb, "B": fk.plan.B}
    for hot in (False, True):
        lab = "hot" if hot else "cold"
        T = {}
        for n in ns:
            T[n] = statistics.median(one(n, hot) for _ in range(a.reps))
        fk.check()
        out[f"{lab}_us"] = {str(n): round(T[n], 2) for n in ns}
        out[f"{lab}_us_per_step"] = {str(n): round(T[n] / n, 3) for n in ns}
        out[f"{lab}_increment_us_per_step"] = {
            f"{p}-{n}": round((T[n] - T[p]) / (n - p), 3) for p, n in zip(ns[:-1], ns[1:])}
    t0 = statistics.median(one(2, False) for _ in range(a.reps))
    out["cold_2step_repeat_us"] = round(t0, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
