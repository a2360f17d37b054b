#!/usr/bin/env python
"""Fixed cost of a short timed region at C96 (GPU): run(K) on a prepared graph,
timed with perf_counter around  sync; run; sync  where the closing sync is
torch.cuda.synchronize (A) or a spin on the stream's query() followed by
torch.cuda.synchronize (B).  Prints median µs/step for K = 20 and 300."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.parallel.layout import TileLayout
    g = CubedSphereGrid(96)
    e = Engine(ShallowWater("tc5"), TileLayout(96, 2, 1, ng=2), grid=g, device="cuda", backend="hip")
    out = {}
    for K in (20, 300):
        ns = NativeStepper(e, use_graph=True, steps_per_graph=K)
        ns.prepare(K)
        ns.run(K)
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        for mode in ("sync", "spin", "event"):
            ts = []
            for _ in range(15):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ns.run(K)
                if mode == "spin":
                    while not s.query():
                        pass
                elif mode == "event":
                    ev = torch.cuda.Event()
                    ev.record(s)
                    while not ev.query():
                        pass
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / K * 1e6)
            out[f"K{K}_{mode}"] = round(statistics.median(ts), 3)
        # launch cost alone: time run(K) without waiting
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ns.run(K)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        out[f"K{K}_host_launch_us"] = round((t1 - t0) * 1e6, 1)
        ns.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
