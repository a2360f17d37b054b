"""The streaming ("march") shallow-water stage (ops/csrc/march_kernel.hip) vs the
PyTorch fp64 reference of the same steps, and vs the block stage kernel (GPU).

Sizes cover a tile narrower than one 60-column strip (both W and E panel-edge
ghosts in one wave), several strips with a partial last strip, row segments
that do and do not divide the tile, and tiles_per_edge 1, 2 and 3 (tile sides
on panel edges and inside a panel)."""
import ctypes

import pytest
import torch

from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.parallel.layout import TileLayout

pytestmark = pytest.mark.gpu


def _relerr(ref, hip):
    a = ref.tiles_view().reshape(4, -1)
    b = hip.tiles_view().reshape(4, -1).double()
    return ((a - b).abs().amax(dim=1) / a.abs().amax(dim=1).clamp_min(1e-30)).max().item()


def _pair(N, t, dtype, block, case="tc5", limiter=2, integ="ssprk3"):
    grid = CubedSphereGrid(N)
    L = TileLayout(N, t, 1, ng=2)
    ref = Engine(ShallowWater(case, limiter=limiter), L, grid=grid, dtype=torch.float64, device="cuda",
                 backend="torch", integrator=integ)
    hip = Engine(ShallowWater(case, limiter=limiter), L, grid=grid, dtype=dtype, device="cuda", backend="hip",
                 integrator=integ, block=block, dt=ref.dt)
    return ref, hip


def test_dpp_wave_shifts():
    from stsphere.ops import native
    L = native.require_native()
    x = torch.arange(64, dtype=torch.float64, device="cuda") + 1.0
    out = torch.full((128,), -1.0, dtype=torch.float64, device="cuda")
    outf = torch.full((128,), -1.0, dtype=torch.float32, device="cuda")
    native.check(L.stsp_dpp_probe(native.ptr(x), native.ptr(out), native.ptr(outf), native.current_stream_handle()),
                 "dpp probe")
    torch.cuda.synchronize()
    want_r = torch.cat([torch.zeros(1, device="cuda", dtype=torch.float64), x[:-1]])
    want_l = torch.cat([x[1:], torch.zeros(1, device="cuda", dtype=torch.float64)])
    assert torch.equal(out[:64], want_r) and torch.equal(out[64:], want_l)
    assert torch.equal(outf[:64].double(), want_r) and torch.equal(outf[64:].double(), want_l)


@pytest.mark.parametrize("N,t,R", [(24, 1, 16), (24, 2, 8), (72, 1, 16), (130, 1, 32), (96, 3, 8), (64, 2, 32),
                                   (25, 1, 8), (50, 2, 4), (27, 1, 16)])
def test_march_fp64_matches_reference(N, t, R):
    ref, hip = _pair(N, t, torch.float64, (64, R))
    ref.step(3)
    hip.step(3)
    torch.cuda.synchronize()
    assert _relerr(ref, hip) < 1e-11


@pytest.mark.parametrize("limiter", [0, 1, 3])
def test_march_limiters(limiter):
    ref, hip = _pair(48, 1, torch.float64, (64, 16), case="tc6", limiter=limiter)
    ref.step(3)
    hip.step(3)
    torch.cuda.synchronize()
    assert _relerr(ref, hip) < 1e-11


@pytest.mark.parametrize("integ", ["euler", "rk4"])
def test_march_integrators(integ):
    ref, hip = _pair(32, 1, torch.float64, (64, 8), integ=integ)
    ref.step(3)
    hip.step(3)
    torch.cuda.synchronize()
    assert _relerr(ref, hip) < 1e-11


@pytest.mark.parametrize("N,t,R", [(72, 1, 16), (48, 2, 8), (96, 3, 8), (250, 1, 8), (25, 1, 8)])
def test_march_fp32_close_to_fp64_reference(N, t, R):
    """fp32 rounding grows with the grid (differences of nearby cells over
    smaller faces), so the gate is the block stage kernel's own fp32 error on
    the same case."""
    ref, hip = _pair(N, t, torch.float32, (64, R))
    blk = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=CubedSphereGrid(N), dtype=torch.float32,
                 device="cuda", backend="hip", block=(16, 16), dt=ref.dt)
    ref.step(3)
    hip.step(3)
    blk.step(3)
    torch.cuda.synchronize()
    e_blk, e_m = _relerr(ref, blk), _relerr(ref, hip)
    assert e_m < 1.5 * e_blk + 2e-5, (e_m, e_blk)
    assert e_blk < 1e-3, e_blk


def test_march_agrees_with_block_kernel():
    N = 96
    grid = CubedSphereGrid(N)
    L = TileLayout(N, 1, 1, ng=2)
    a = Engine(ShallowWater("tc5"), L, grid=grid, device="cuda", backend="hip", block=(8, 8))
    b = Engine(ShallowWater("tc5"), L, grid=grid, device="cuda", backend="hip", block=(64, 16), dt=a.dt)
    a.step(6)
    b.step(6)
    torch.cuda.synchronize()
    d = (a.tiles_view() - b.tiles_view()).abs().amax().item()
    assert d <= 1e-12 * a.tiles_view().abs().amax().item()


def test_march_never_uses_a_corner_ghost():
    g = CubedSphereGrid(48)
    L = TileLayout(48, 2, 1, ng=2)
    a = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", block=(64, 8))
    b = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", block=(64, 8), dt=a.dt)
    b.poison_corners()
    a.step(4)
    b.step(4)
    torch.cuda.synchronize()
    assert torch.isfinite(b.tiles_view()).all()
    assert torch.equal(a.tiles_view(), b.tiles_view())


def test_march_refuses_ppm():
    g = CubedSphereGrid(24)
    L = TileLayout(24, 1, 1, ng=3)
    with pytest.raises(ValueError):
        Engine(ShallowWater("tc5", limiter=4), L, grid=g, device="cuda", backend="hip", block=(64, 16))
