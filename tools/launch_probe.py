#!/usr/bin/env python
"""Host-timed launch forms of the fused multi-step kernel, timed exactly like
bench.py's timed region (synchronize; K steps; synchronize) so the fixed cost
per timed run is visible: graph replay of one K-step launch (the bench's path),
the C++ runtime's eager launch, and a direct launch through ctypes.  One JSON
line; medians over --reps repetitions.

    python tools/launch_probe.py --N 96 --t 2 --steps 20 --reps 30
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
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--t", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.parallel.layout import TileLayout
    L = TileLayout(a.N, a.t, 1, ng=2)
    e = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(a.N), dtype=torch.float64, device="cuda", backend="hip")
    fk = FusedKernel(e)
    K = a.steps
    r = NativeStepper(e, use_graph=True, steps_per_graph=K, fused=fk, steps_per_launch=K)
    r.prepare(K)
    cur = torch.cuda.current_stream()

    def timed(fn, idle=0.0):
        ts = []
        for _ in range(a.reps):
            if idle:
                time.sleep(idle)      # GPU idle before the timed region (as after the bench's warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6 / K)
        return statistics.median(ts), min(ts)

    out = {"N": a.N, "t": a.t, "steps": K, "blocks": fk.plan.nb}
    rd = NativeStepper(e, use_graph=True, steps_per_graph=K, fused=fk, steps_per_launch=K, direct=True)
    rd.prepare(K)
    forms = {
        "graph_replay": lambda: r.run(K),
        "cxx_eager": lambda: r._run_native(K),
        "ctypes_direct": lambda: fk.launch(0, int(cur.cuda_stream), nsteps=K),
        "runner_direct": lambda: rd.run(K),
    }
    for idle in (0.0, 0.002, 0.05):
        for name, fn in forms.items():
            fn()
            torch.cuda.synchronize()
            med, best = timed(fn, idle)
            tag = name if not idle else f"{name}_idle{int(idle * 1e3)}ms"
            out[tag + "_us_per_step"] = round(med, 3)
            out[tag + "_best"] = round(best, 3)
    # an empty timed region: the synchronize pair alone
    med, best = timed(lambda: None)
    out["empty_region_us_total"] = round(med * K, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
