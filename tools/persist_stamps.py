"""Per-stage phase timeline of the persistent step kernel (stepdbg library
variant, STSP_VARIANT=stepdbg): window wait, compute, skew across blocks.
Prints a summary and writes the raw stamps to gpurun_out/persist_stamps.json."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("STSP_VARIANT", "stepdbg")
import numpy as np
import torch
from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.parallel.layout import TileLayout
from stsphere.ops.persistent import PersistentStepper

N = int(sys.argv[1]) if len(sys.argv) > 1 else 96
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
exch = sys.argv[3] if len(sys.argv) > 3 else "uncached"
g = CubedSphereGrid(N)
e = Engine(ShallowWater("tc5"), TileLayout(N, 2, 1, ng=2), grid=g, device="cuda", backend="hip", block=(16, 16))
ps = PersistentStepper(e, timeout_s=1.0, max_steps_per_launch=steps, exchange=exch)
ps.run(steps)          # warm
ps.dbg.zero_()
torch.cuda.synchronize()
import time
t0 = time.perf_counter()
ps.run(steps)
torch.cuda.synchronize()
print("wall us/step", (time.perf_counter() - t0) / steps * 1e6)
ps.check()
nb = e.compute.nblocks
st = ps.dbg[4096:4096 + nb * 128].view(nb, 16, 8).cpu().numpy().astype(np.float64) * 10.0   # ns
S = min(16, 3 * steps)
t0 = st[:, 0, 0].min()
st = st - t0
out = {"nblocks": nb, "stages": []}
for s in range(S):
    w = st[:, s, 1] - st[:, s, 0]
    c = st[:, s, 2] - st[:, s, 1]
    rec = {"s": s, "start_min_ns": float(st[:, s, 0].min()), "start_max_ns": float(st[:, s, 0].max()),
           "window_done_max_ns": float(st[:, s, 1].max()), "flux_done_max_ns": float(st[:, s, 2].max()),
           "wait_mean_ns": float(w.mean()), "wait_max_ns": float(w.max()),
           "compute_mean_ns": float(c.mean()), "compute_max_ns": float(c.max())}
    own_upd = st[:, s, 4] - st[:, s, 2]
    issue = st[:, s, 5] - st[:, s, 4]
    drain = st[:, s, 7] - st[:, s, 5]
    wexit = st[:, s, 6] - st[:, s, 0]
    bar = st[:, s, 1] - st[:, s, 6]
    rec.update({"own_update_ns": float(own_upd.mean()), "store_issue_ns": float(issue.mean()),
                "store_drain_ns": float(drain.mean()), "wave0_wait_ns": float(wexit.mean()),
                "barrier_after_wave0_ns": float(bar.mean())})
    if s + 1 < S:
        u = st[:, s + 1, 0] - st[:, s, 2]
        rec["update_mean_ns"] = float(u.mean())
        rec["update_max_ns"] = float(u.max())
    out["stages"].append(rec)
    print(json.dumps(rec))
os.makedirs("gpurun_out", exist_ok=True)
with open(f"gpurun_out/persist_stamps_{os.environ['STSP_VARIANT']}_{exch}.json", "w") as f:
    json.dump(out, f, indent=1)
