"""Long-run GPU oracle checks: one simulated day of Williamson TC5 (zonal flow
over the mountain, SURVEY.md 4 "TC5 error norms") at C48 through every HIP step
path, against the PyTorch fp64 reference stepping the same dt on the GPU.

Short tests (2-3 steps) pin each kernel to the oracle at 1e-11; these bound the
drift that per-step roundoff (panel edges, cube corners, the band / march seam
of the pipelined step) can accumulate over a day: ~100 steps."""
import math

import pytest
import torch

from stsphere.engine import Engine
from stsphere.models.geometry import DAY, CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.parallel.layout import TileLayout

pytestmark = pytest.mark.gpu

N = 48


def _relerr(ref, hip):
    a = ref.tiles_view().reshape(4, -1)
    b = hip.tiles_view().reshape(4, -1).double()
    return ((a - b).abs().amax(dim=1) / a.abs().amax(dim=1).clamp_min(1e-30)).max().item()


_REF = {}


def _oracle(t):
    """fp64 torch reference after one day (cached per tiling)."""
    if t not in _REF:
        grid = CubedSphereGrid(N)
        ref = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=grid, dtype=torch.float64, device="cuda",
                     backend="torch")
        steps = math.ceil(DAY / ref.dt)
        ref.step(steps)
        torch.cuda.synchronize()
        _REF[t] = (ref, steps)
    return _REF[t]


def _hip(t, dtype, dt, **kw):
    return Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=CubedSphereGrid(N), dtype=dtype,
                  device="cuda", backend="hip", dt=dt, **kw)


@pytest.mark.parametrize("t,B", [(1, 16), (2, 6)])
def test_fused_one_day_fp64(t, B):
    from stsphere.ops.fused import FusedKernel
    ref, steps = _oracle(t)
    hip = _hip(t, torch.float64, ref.dt)
    fk = FusedKernel(hip, B=B)
    fk.step(steps)
    torch.cuda.synchronize()
    fk.check()
    err = _relerr(ref, hip)
    print(f"fused B={B} t={t}: {steps} steps, max rel diff {err:.3e}")
    assert err < 1e-11


def test_streaming_stage_one_day_fp64():
    ref, steps = _oracle(1)
    hip = _hip(1, torch.float64, ref.dt, block=(64, 8))
    hip.step(steps)
    torch.cuda.synchronize()
    err = _relerr(ref, hip)
    print(f"streaming stage 64x8: {steps} steps, max rel diff {err:.3e}")
    assert err < 1e-11


def test_pipelined_march_one_day_fp64():
    from stsphere.ops.march3 import March3Step
    ref, steps = _oracle(1)
    hip = _hip(1, torch.float64, ref.dt)
    March3Step(hip, rows=16).step(steps)
    torch.cuda.synchronize()
    err = _relerr(ref, hip)
    print(f"pipelined march: {steps} steps, max rel diff {err:.3e}")
    assert err < 1e-11


def test_one_day_fp32_drift():
    """fp32 stays within a fixed bound of the fp64 oracle over a day on the
    fused and the pipelined paths (no runaway from the panel edges)."""
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.march3 import March3Step
    ref, steps = _oracle(1)
    a = _hip(1, torch.float32, ref.dt)
    FusedKernel(a, B=16).step(steps)
    b = _hip(1, torch.float32, ref.dt)
    March3Step(b, rows=16).step(steps)
    torch.cuda.synchronize()
    ea, eb = _relerr(ref, a), _relerr(ref, b)
    print(f"fp32 one day: fused {ea:.3e}, pipelined march {eb:.3e}")
    assert ea < 2e-4 and eb < 2e-4
