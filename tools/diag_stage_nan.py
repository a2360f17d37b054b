import sys, torch
sys.path.insert(0, '/root/repo')
sys.path.insert(0, '.')
from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.parallel.layout import TileLayout
for t in (1, 2):
    for lim in (3, 2):
        grid = CubedSphereGrid(24)
        L = TileLayout(24, t, 1, ng=2)
        mk = lambda: ShallowWater("tc6", limiter=lim)
        ref = Engine(mk(), L, grid=grid, dtype=torch.float64, device="cuda", backend="torch")
        hip = Engine(mk(), L, grid=grid, dtype=torch.float64, device="cuda", backend="hip", block=(16, 16))
        hip.dt = ref.dt
        for k in range(4):
            ref.step(1); hip.step(1); torch.cuda.synchronize()
            a = ref.tiles_view(); b = hip.tiles_view()
            na, nb = int(torch.isnan(a).sum()), int(torch.isnan(b).sum())
            d = float((a - b).abs().max())
            print(f"t={t} lim={lim} step {k}: nan ref {na} hip {nb} maxdiff {d:.3e}", flush=True)
            if nb:
                idx = torch.nonzero(torch.isnan(b))[:5].tolist()
                print("   first nan (f, tile, j, i):", idx, flush=True)
                break
