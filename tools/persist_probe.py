"""Persistent-kernel phase split (diag build): per stage, cycles in the stage
body, in the store drain + barrier, and waiting for neighbour flags."""
import json, os, sys
os.environ["STSP_VARIANT"] = "diag"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.ops import native
from stsphere.ops.persistent import PersistentStepper
from stsphere.parallel.layout import TileLayout

N = int(sys.argv[1]) if len(sys.argv) > 1 else 96
e = Engine(ShallowWater("tc5"), TileLayout(N, 2, 1, ng=2), grid=CubedSphereGrid(N), device="cuda", backend="hip")
ps = PersistentStepper(e)
stamps = torch.zeros(e.compute.nblocks * 256, dtype=torch.int64, device="cuda")   # [block][16 waves][16] per-wave stamps; [block][0..2] sums
ps._descs[0].stamps = native.ptr(stamps)
steps = 100
ps.run(5)
torch.cuda.synchronize()
t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
t0.record(); ps.run(steps); t1.record(); torch.cuda.synchronize()
ps.check()
st = stamps.view(-1, 256)[:, :8].cpu().numpy().astype(float)
nst = steps * 3
print(json.dumps({"us_per_step": t0.elapsed_time(t1) * 1e3 / steps,
                  "cycles_per_stage_median": {"body": float(np.median(st[:, 0]) / nst),
                                              "drain+barrier": float(np.median(st[:, 1]) / nst),
                                              "wait": float(np.median(st[:, 2]) / nst)},
                  "wait_max_block": float(st[:, 2].max() / nst)}, indent=1))
