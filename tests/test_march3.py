"""The pipelined streaming SSP-RK3 step (ops/csrc/march3_kernel.hip + the band
launches of the stage kernel, ops/march3.py) vs the PyTorch fp64 reference of
the same steps (GPU), and its host-side band / strip bookkeeping (CPU).

Sizes cover one strip per tile and several (a partial last strip), segments
that do and do not divide the tile, tiles whose size is not a multiple of the
8x8 band blocks (n % 8 = 2, 6), and tiles_per_edge 1, 2 and 3 (tile sides on
panel edges and inside a panel)."""
import numpy as np
import pytest
import torch

from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.ops.march3 import M3_COLS, band_blocks
from stsphere.parallel.layout import TileLayout


# ---- CPU: band blocks and strip / segment coverage ------------------------------
@pytest.mark.parametrize("n", [24, 30, 48, 50, 57, 90, 120, 180, 360, 720])
def test_band_blocks_cover_the_cells_the_march_leaves(n):
    """Every cell within 4 of a tile edge (where the march computes no stage 3,
    and no stage 2 within 2) lies in a band block, and every cell a band block
    reads (block + ring of 2) is within D - 1 of the tile edge, so the march
    stored its stage-1 / stage-2 value."""
    T = 2
    ids, D = band_blocks(n, T)
    nbx = -(-n // 8)
    cover = np.zeros((n, n), bool)
    reach = np.zeros((n + 4, n + 4), bool)
    for b in ids[ids < nbx * nbx]:
        yb, xb = divmod(int(b), nbx)
        cover[yb * 8:min(n, yb * 8 + 8), xb * 8:min(n, xb * 8 + 8)] = True
        reach[yb * 8:min(n, yb * 8 + 8) + 4, xb * 8:min(n, xb * 8 + 8) + 4] = True
    c = np.arange(n)
    dist = np.minimum(np.minimum(c[:, None], n - 1 - c[:, None]), np.minimum(c[None, :], n - 1 - c[None, :]))
    assert cover[dist < 4].all()
    reach = reach[2:n + 2, 2:n + 2]
    assert (dist[reach] < D).all()
    assert len(ids) == T * len(ids[ids < nbx * nbx])
    assert len(set(ids.tolist())) == len(ids)


@pytest.mark.parametrize("n", [24, 30, 50, 57, 90, 120, 180, 720])
@pytest.mark.parametrize("R", [16, 32, 64])
def test_march3_strips_and_segments_partition_the_tile(n, R):
    """Mirror of march3_kernel's ownership: the strips' owned columns and the
    segments' owned rows partition the tile, every owned column is inside the
    strip's stage-1 lanes (2..61), the stage-3 columns [4, n - 4) inside its
    stage-3 lanes (6..57), and the stage rows stay inside the padded tile."""
    ncs = -(-(n - 8) // M3_COLS)
    nrs = -(-(n - 8) // R)
    seen = np.zeros(n, int)
    for cs in range(ncs):
        olo = 0 if cs == 0 else cs * M3_COLS + 4
        ohi = n if cs == ncs - 1 else cs * M3_COLS + 4 + M3_COLS
        seen[olo:ohi] += 1
        x = cs * M3_COLS + np.arange(64) - 2
        assert x[2] <= olo and x[61] >= ohi - 1
        s3 = [v for v in range(olo, ohi) if 4 <= v < n - 4]
        if s3:
            assert x[6] <= min(s3) and x[57] >= max(s3)
    assert (seen == 1).all()
    rows = np.zeros(n, int)
    for rs in range(nrs):
        ys = 4 + rs * R
        ye = min(ys + R, n - 4)
        assert ys < ye
        rlo = 0 if rs == 0 else ys
        rhi = n if rs == nrs - 1 else ye
        rows[rlo:rhi] += 1
        assert ys - 6 >= -2 and ye + 5 <= n + 1     # input rows inside the padded tile (ng = 2)
        assert ys - 4 <= rlo and ye + 4 >= rhi      # stage-1 rows cover the owned rows
    assert (rows == 1).all()


def test_march3_refuses_what_it_cannot_run():
    from stsphere.ops.march3 import march3_unsupported
    L = TileLayout(48, 1, 1, ng=2)
    e = Engine(ShallowWater("tc5"), L, dtype=torch.float64, device="cpu", backend="torch")
    assert "backend" in march3_unsupported(e)


# ---- GPU: numerics -----------------------------------------------------------------
def _relerr(ref, hip):
    a = ref.tiles_view().reshape(4, -1)
    b = hip.tiles_view().reshape(4, -1).double()
    return ((a - b).abs().amax(dim=1) / a.abs().amax(dim=1).clamp_min(1e-30)).max().item()


def _pair(N, t, dtype, case="tc5", limiter=2):
    grid = CubedSphereGrid(N)
    L = TileLayout(N, t, 1, ng=2)
    ref = Engine(ShallowWater(case, limiter=limiter), L, grid=grid, dtype=torch.float64, device="cuda",
                 backend="torch")
    hip = Engine(ShallowWater(case, limiter=limiter), L, grid=grid, dtype=dtype, device="cuda", backend="hip",
                 dt=ref.dt)
    return ref, hip


@pytest.mark.gpu
@pytest.mark.parametrize("N,t,R", [(48, 1, 16), (50, 1, 32), (60, 2, 16), (96, 2, 32), (130, 1, 64), (120, 1, 16),
                                   (90, 3, 16), (144, 1, 32)])
def test_march3_fp64_matches_reference(N, t, R):
    from stsphere.ops.march3 import March3Step
    ref, hip = _pair(N, t, torch.float64)
    m3 = March3Step(hip, rows=R)
    ref.step(3)
    m3.step(3)
    torch.cuda.synchronize()
    assert torch.isfinite(hip.tiles_view()).all()
    assert _relerr(ref, hip) < 1e-11


@pytest.mark.gpu
@pytest.mark.parametrize("limiter", [0, 1, 3])
def test_march3_limiters(limiter):
    from stsphere.ops.march3 import March3Step
    ref, hip = _pair(64, 1, torch.float64, case="tc6", limiter=limiter)
    m3 = March3Step(hip, rows=16)
    ref.step(3)
    m3.step(3)
    torch.cuda.synchronize()
    assert _relerr(ref, hip) < 1e-11


@pytest.mark.gpu
@pytest.mark.parametrize("N,t", [(96, 1), (72, 2)])
def test_march3_fp32_close_to_fp64_reference(N, t):
    """fp32 rounding grows with the grid: the gate is the block stage
    kernel's own fp32 error on the same case (as tests/test_march.py)."""
    from stsphere.ops.march3 import March3Step
    ref, hip = _pair(N, t, torch.float32)
    blk = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=CubedSphereGrid(N), dtype=torch.float32,
                 device="cuda", backend="hip", block=(16, 16), dt=ref.dt)
    m3 = March3Step(hip, rows=32)
    ref.step(3)
    m3.step(3)
    blk.step(3)
    torch.cuda.synchronize()
    e_blk, e_m = _relerr(ref, blk), _relerr(ref, hip)
    assert e_m < 1.5 * e_blk + 2e-5, (e_m, e_blk)
    assert e_blk < 1e-3, e_blk


@pytest.mark.gpu
def test_march3_native_stepper_graph_equals_eager_and_conserves_mass():
    """NativeStepper(march3=...) replays the two-step op list from a hipGraph:
    bitwise equal to the eager pipelined steps, mass conserved to round-off."""
    from stsphere.ops.march3 import March3Step
    from stsphere.ops.native_runtime import NativeStepper
    N = 96
    grid = CubedSphereGrid(N)
    L = TileLayout(N, 1, 1, ng=2)
    a = Engine(ShallowWater("tc5"), L, grid=grid, dtype=torch.float64, device="cuda", backend="hip")
    b = Engine(ShallowWater("tc5"), L, grid=grid, dtype=torch.float64, device="cuda", backend="hip", dt=a.dt)
    m0 = a.diagnostics()["mass"]
    ma = March3Step(a, rows=32)
    ma.step(6)
    r = NativeStepper(b, use_graph=True, steps_per_graph=6, march3=March3Step(b, rows=32))
    r.prepare(6)
    r.run(6)
    torch.cuda.synchronize()
    assert r.stats["graph_steps"] == 6 and r.stats["eager_steps"] == 0
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert abs(b.diagnostics()["mass"] - m0) <= 1e-12 * abs(m0)
    r.close()


@pytest.mark.gpu
def test_march3_band_launches_finish_the_edges():
    """Without the two band launches the cells within 4 of a tile edge keep the
    old output (poisoned with NaN here) and the march's own cells are already
    final: the band launches are what completes the step."""
    import ctypes
    from stsphere.ops import native
    from stsphere.ops.march3 import March3Step
    ref, hip = _pair(48, 1, torch.float64)
    m3 = March3Step(hip, rows=16)
    dst = torch.full_like(hip.pool[0], float("nan"))
    d, m, band = m3.step_descs(hip.pool[0], dst)
    L = native.require_native()
    native.check(L.stsp_march3_launch(1, 16, ctypes.byref(d), ctypes.byref(m), native.current_stream_handle()),
                 "march3")
    ref.step(1)
    torch.cuda.synchronize()
    got = hip.interior(dst)
    want = ref.tiles_view()
    n = 48
    c = torch.arange(n, device="cuda")
    dist = torch.minimum(torch.minimum(c[:, None], n - 1 - c[:, None]), torch.minimum(c[None, :], n - 1 - c[None, :]))
    inner = dist >= 4
    assert torch.isnan(got[:, :, ~inner]).all()
    err = ((got[:, :, inner] - want[:, :, inner]).abs().amax() / want.abs().amax()).item()
    assert err < 1e-11
