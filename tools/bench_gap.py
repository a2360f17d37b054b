"""Where the bench's fixed cost per timed region goes (C96 fused, one GPU).

bench.py times ONE ``runner.run(K)`` between two synchronisations.  This
probe builds the same engine and runner and reports, per K:
  host_us      host perf_counter around sync / run(K) / sync (the bench's clock)
  event_us     hipEvent pair around run(K) on the stream (GPU start to end)
  fit          least-squares  T(K) = a + b K  over K in KS, for both clocks
and back-to-back regions (no sync between launches), which hide the launch
latency.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--t", type=int, default=2)
    ap.add_argument("--ks", default="2,4,10,20,40,100")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--sync", default="spin", choices=["spin", "auto"])
    a = ap.parse_args()
    if a.sync == "spin":
        from stsphere.ops import native
        rc = native.load(build_if_missing=False).stsp_schedule_spin(0)
        print("schedule_spin rc", rc, file=sys.stderr)
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.fused import FusedKernel, fused_block
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.parallel.layout import TileLayout

    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    L = TileLayout(a.N, a.t, 1, ng=2)
    eng = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(a.N), dtype=torch.float64, device=dev, backend="hip")
    fk = FusedKernel(eng, B=fused_block(L.n, 6 * a.t * a.t, cus))
    ks = [int(k) for k in a.ks.split(",")]
    out = {"sync": a.sync, "N": a.N, "t": a.t, "B": fk.plan.B, "blocks": fk.plan.nb, "per_K": {}}
    runners = {}
    for k in ks:
        r = NativeStepper(eng, use_graph=True, fused=fk, steps_per_launch=k, direct=True)
        r.prepare(k)
        r.run(k)
        torch.cuda.synchronize()
        runners[k] = r
    for k in ks:
        r = runners[k]
        host, ev = [], []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            r.run(k)
            e1.record()
            torch.cuda.synchronize()
            host.append((time.perf_counter() - t0) * 1e6)
            ev.append(e0.elapsed_time(e1) * 1e3)
        # host cost of issuing run(k) (no sync) and of a synchronize on an idle GPU
        enq, idle = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.run(k)
            enq.append((time.perf_counter() - t0) * 1e6)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            idle.append((time.perf_counter() - t0) * 1e6)
        # back to back: 10 regions, one sync
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            r.run(k)
        torch.cuda.synchronize()
        b2b = (time.perf_counter() - t0) * 1e6 / 10
        out["per_K"][k] = {"host_us_min": min(host), "host_us_med": float(np.median(host)),
                           "event_us_min": min(ev), "event_us_med": float(np.median(ev)),
                           "b2b_host_us": b2b, "enqueue_us_med": float(np.median(enq)),
                           "idle_sync_us_med": float(np.median(idle))}
        print(k, out["per_K"][k], file=sys.stderr, flush=True)
    K = np.array(ks, dtype=float)
    for key in ("host_us_min", "event_us_min", "b2b_host_us"):
        y = np.array([out["per_K"][k][key] for k in ks])
        b, a0 = np.polyfit(K, y, 1)
        out[f"fit_{key}"] = {"fixed_us": float(a0), "per_step_us": float(b)}
    fk.check()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
