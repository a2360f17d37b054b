"""Persistent step kernel vs launch-per-stage: max |diff| per config, and
where the first differences sit (tile, row, col) after a few steps."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('STSP_STEP_DEBUG', '1')
import torch
from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.models.advection import Advection
from stsphere.parallel.layout import TileLayout
from stsphere.ops.persistent import PersistentStepper

import json
cfgs = [tuple(c) for c in json.loads(sys.argv[1])] if len(sys.argv) > 1 else [
    (96, 2, (16, 16), 1), (96, 2, (16, 16), 2), (96, 2, (16, 8), 1), (48, 2, (8, 8), 1), (24, 2, (16, 16), 1),
    (24, 2, (8, 8), 1), (96, 2, (16, 16), 7)]
for N, t, blk, steps in cfgs:
    blk = tuple(blk)
    g = CubedSphereGrid(N)
    L = TileLayout(N, t, 1, ng=2)
    a = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", block=blk)
    b = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", dt=a.dt, block=blk)
    ps = PersistentStepper(b, timeout_s=1.0, max_steps_per_launch=100)
    a.step(steps)
    ps.run(steps)
    torch.cuda.synchronize()
    err = int(ps.err[0].item())
    d = (a.tiles_view() - b.tiles_view()).abs()
    m = float(d.max())
    line = f"N={N} t={t} blk={blk} steps={steps} err={err} maxdiff={m:.3e}"
    if m > 0:
        nz = torch.nonzero(d[0] > 0)
        line += f" ncells={nz.shape[0]} first={nz[:6].tolist()}"
        e1 = float((a.pool[0] - b.pool[0]).abs().max())
        line += f" pooldiff={e1:.3e}"
    print(line, flush=True)
    if err and ps.dbg is not None:
        dd = ps.dbg.cpu().tolist()
        print("  timeouts recorded:", dd[0])
        for i in range(min(dd[0], 12)):
            r = dd[8 + 8 * i: 16 + 8 * i]
            print("  bid=%d s=%d pa=%d want=%d seen=%d wly=%d wlx=%d hwid=%x" % tuple(r))
