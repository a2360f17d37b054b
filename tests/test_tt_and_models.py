"""TT numerics (S10), roofline model (S14), visualisation (S13)."""
import math
import os

import numpy as np
import pytest
import torch

from stsphere.models import tt
from stsphere.models.geometry import CubedSphereGrid
from stsphere.utils import roofline


def test_tt_svd_roundtrip_and_accuracy():
    torch.manual_seed(0)
    x = torch.randn(4, 5, 6, 3, dtype=torch.float64)
    cores = tt.tt_svd(x, eps=1e-12)
    assert torch.allclose(tt.tt_full(cores), x, atol=1e-10)
    # low-rank tensor compresses exactly
    a, b, c = (torch.randn(n, dtype=torch.float64) for n in (8, 9, 10))
    y = torch.einsum("i,j,k->ijk", a, b, c) + 2 * torch.einsum("i,j,k->ijk", b[:8], a[:8].repeat(2)[:9], c)
    cy = tt.tt_svd(y, eps=1e-12)
    assert max(tt.tt_ranks(cy)) <= 2
    assert torch.allclose(tt.tt_full(cy), y, atol=1e-10)


def test_tt_arithmetic_and_rounding():
    torch.manual_seed(1)
    x = torch.randn(3, 4, 5, dtype=torch.float64)
    y = torch.randn(3, 4, 5, dtype=torch.float64)
    cx, cy = tt.tt_svd(x), tt.tt_svd(y)
    s = tt.tt_add(cx, tt.tt_scale(cy, 2.0))
    assert torch.allclose(tt.tt_full(s), x + 2 * y, atol=1e-10)
    assert abs(float(tt.tt_dot(cx, cy)) - float((x * y).sum())) < 1e-9
    assert abs(tt.tt_norm(cx) - float(x.norm())) < 1e-9
    r = tt.tt_round(tt.tt_add(cx, cx), eps=1e-12)
    assert torch.allclose(tt.tt_full(r), 2 * x, atol=1e-9) and tt.tt_ranks(r) == tt.tt_ranks(cx)


def test_qtt_smooth_field_low_rank():
    n = 256
    xx = torch.linspace(0, 1, n, dtype=torch.float64)
    f = torch.sin(3 * xx)[:, None] * torch.cos(2 * xx)[None, :] + torch.exp(-((xx[:, None] - .5) ** 2 + (xx[None] - .5) ** 2) * 8)
    t = tt.qtt_reshape(f)
    assert torch.equal(tt.qtt_unreshape(t), f)
    cores = tt.tt_svd(t, eps=1e-6)
    assert tt.tt_storage(cores) < f.numel() / 4
    assert float((tt.qtt_unreshape(tt.tt_full(cores)) - f).norm() / f.norm()) < 1e-6


def test_low_rank_diffusion_matches_dense():
    N = 48
    solver = tt.LowRankDiffusion(N, kappa=1.0, eps=1e-12, max_rank=20)
    x = torch.linspace(0, 1, N + 2, dtype=torch.float64)[1:-1]
    U = torch.sin(math.pi * x)[:, None] * torch.sin(2 * math.pi * x)[None, :] + \
        0.3 * torch.sin(3 * math.pi * x)[:, None] * torch.sin(math.pi * x)[None, :]
    lr = tt.LowRankField.from_dense(U, eps=1e-14)
    assert lr.rank == 2
    dt = 0.5 * solver.dt_max
    dense = U.clone()
    for _ in range(50):
        lr = solver.step(lr, dt)
        dense = solver.dense_step(dense, dt)
    assert lr.rank <= 4
    assert float((lr.dense() - dense).norm() / dense.norm()) < 1e-10


def test_compress_cubed_sphere_field():
    g = CubedSphereGrid(32)
    from stsphere.models.initial_conditions import williamson_tc2
    h, _, _ = williamson_tc2(g.centers())
    rep = tt.compress_cubed_sphere(h, eps=1e-6, qtt=False)   # panel rank 4 at C32
    assert all(r["rel_error"] < 1e-5 for r in rep)
    assert np.mean([r["compression"] for r in rep]) > 3 and max(max(r["ranks"]) for r in rep) <= 6


def test_roofline_reproduces_slide19():
    assert abs(roofline.TPU_V4_CLASS.ridge - 305.6) < 0.1
    assert abs(roofline.fv_plr_cell_rate(roofline.TPU_V4_CLASS) - 2.586e8) < 1e6
    table = {c["r"]: c for c in roofline.tt_savings_table()}
    for r, (fl, mem, ai, tot) in {10: (8.3, 5.3, 17.5, 144), 16: (2.0, 2.0, 28, 56), 20: (1.05, 1.3, 35, 35),
                                  30: (0.31, 0.59, 52, 16)}.items():
        c = table[r]
        for got, want in ((c["flop_reduction"], fl), (c["memory_reduction"], mem), (c["tt_ai"], ai),
                          (c["total_savings"], tot)):
            assert abs(got / want - 1) < 0.12, (r, got, want)


def test_viz_products(tmp_path):
    from stsphere.utils import viz
    from stsphere.models.initial_conditions import cosine_bell, lima_flag
    g = CubedSphereGrid(12)
    bell = cosine_bell(g.centers())
    assert os.path.getsize(viz.latlon_band(bell, g, str(tmp_path / "band.png"))) > 1000
    assert os.path.getsize(viz.sphere_plot(lima_flag(12), g, str(tmp_path / "s.png"), log=True)) > 1000
    assert os.path.getsize(viz.six_panel(bell, bell, str(tmp_path / "six.png"))) > 1000
    assert os.path.getsize(viz.mesh_plot(g, str(tmp_path / "mesh.png"))) > 1000


def _cube_field(N):
    x = (torch.arange(N, dtype=torch.float64) + 0.5) / N
    return torch.stack([torch.outer(torch.sin(math.pi * x * (p + 1) / 3), torch.cos(math.pi * x * (p % 3 + 1) / 2))
                        + (1.0 if p == 2 else 0.0) for p in range(6)])


def test_cube_low_rank_diffusion_matches_dense_six_panel_step():
    """Factored diffusion on the six panels, coupled through the factored cube
    halo, equals the dense six-panel five-point step (same ghost map) to the
    truncation tolerance, conserves the total, and keeps low ranks."""
    N = 32
    m = tt.CubedSphereLowRankDiffusion(N, eps=1e-12)
    assert all(m.nbr[p][s] is not None and m.nbr[p][s] != p for p in range(6) for s in range(4))
    # the neighbour relation is symmetric: q borders p on some side iff p borders q
    for p in range(6):
        for s in range(4):
            assert p in m.nbr[m.nbr[p][s]]
    U = _cube_field(N)
    F, D = m.to_factored(U), U.clone()
    dt = 0.8 * m.dt_max
    for _ in range(20):
        F, D = m.step(F, dt), m.dense_step(D, dt)
    R = m.to_dense(F)
    assert float((R - D).norm() / D.norm()) < 1e-10
    assert abs(float(R.sum()) / float(U.sum()) - 1) < 1e-12
    assert max(f.rank for f in F) < N


def test_cube_low_rank_halo_is_the_dense_halo():
    """Ghost strips gathered from the factors are the dense ghost cells."""
    N = 16
    m = tt.CubedSphereLowRankDiffusion(N, eps=1e-14)
    U = _cube_field(N) + 0.1 * torch.rand(6, N, N, dtype=torch.float64)
    F = m.to_factored(U)
    P = torch.zeros((6, N + 2, N + 2), dtype=torch.float64)
    P[:, 1:-1, 1:-1] = m.to_dense(F)
    P.reshape(-1)[m._ddst] = P.reshape(-1)[m._dsrc]
    for p in range(6):
        g = m.ghosts(F, p)
        assert torch.allclose(g[0], P[p, 1:-1, 0], atol=1e-12)
        assert torch.allclose(g[1], P[p, 1:-1, -1], atol=1e-12)
        assert torch.allclose(g[2], P[p, 0, 1:-1], atol=1e-12)
        assert torch.allclose(g[3], P[p, -1, 1:-1], atol=1e-12)


@pytest.mark.parametrize("substeps", [2, 3])
def test_low_rank_diffusion_substeps_exact_between_recompressions(substeps):
    """substeps > 1: the factors grow exactly ([A, c D A], [B + c D B, B] per
    step) and are recompressed once per call; equal to dense stepping."""
    N = 64
    x = torch.linspace(0, 1, N + 2, dtype=torch.float64)[1:-1]
    U = torch.outer(torch.sin(math.pi * x), torch.sin(2 * math.pi * x)) + \
        0.3 * torch.outer(torch.sin(3 * math.pi * x), torch.sin(math.pi * x))
    s = tt.LowRankDiffusion(N, eps=1e-12, substeps=substeps)
    dt = 0.5 * s.dt_max
    F, D = tt.LowRankField.from_dense(U, 1e-12), U.clone()
    for _ in range(12 // substeps):
        F = s.step(F, dt)
    for _ in range(12):
        D = s.dense_step(D, dt)
    assert float((F.dense() - D).norm() / D.norm()) < 1e-13
    assert F.rank == 2


def test_cholqr3_orthonormal_and_exact_cpu():
    """Shifted CholeskyQR3 (models/tt.py::cholqr3): Q orthonormal and X = Q R to
    working precision, also for exactly rank-deficient factors (repeated
    columns, as in the expanded factors of a step)."""
    from stsphere.models import tt
    g = torch.Generator().manual_seed(1)
    A = torch.randn(400, 6, dtype=torch.float64, generator=g)
    X = torch.cat([A, 0.3 * A[:, :2], torch.randn(400, 4, dtype=torch.float64, generator=g)], 1)   # rank 10 of 12
    Q, R, info = tt.cholqr3(X)
    assert int(info.abs().sum()) == 0
    assert float((Q @ R - X).norm() / X.norm()) < 1e-14
    # full-rank factor: orthonormal to machine precision
    Q2, R2, _ = tt.cholqr3(torch.randn(400, 12, dtype=torch.float64, generator=g))
    assert float((Q2.T @ Q2 - torch.eye(12, dtype=torch.float64)).abs().max()) < 1e-13


def test_recompress_many_machine_precision_cpu():
    """The CholeskyQR3 recompression keeps a step's product to ~1e-15, where the
    Gram/eigen route stops near sqrt(eps)."""
    from stsphere.models import tt
    N = 256
    x = torch.linspace(0, 1, N, dtype=torch.float64)
    U = torch.exp(-((x[:, None] - 0.4) ** 2 + (x[None, :] - 0.6) ** 2) / 0.02) + torch.sin(3 * x[:, None]) * torch.cos(2 * x[None, :])
    lr = tt.LowRankField.from_dense(U, eps=1e-15)
    s = tt.LowRankDiffusion(N, eps=1e-14)
    c = 0.2 * s.h ** 2
    A = torch.cat([lr.A, c * (s.D @ lr.A), c * lr.A], 1)
    B = torch.cat([lr.B, lr.B, s.D @ lr.B], 1)
    f, = tt.recompress_many([(A, B)], 1e-14, None)
    dense = A @ B.T
    assert float((f.dense() - dense).norm() / dense.norm()) < 1e-13


def test_factored_advection_matches_dense_operator_cpu():
    """CubedSphereLowRankAdvection (models/tt.py): the factored SSP-RK3 step of
    TC1 advection with the sphere metric equals the dense N x N six-panel step
    of the same operator to the truncation tolerance, and conserves mass."""
    from stsphere.models import tt
    from stsphere.models import initial_conditions as ic
    m = tt.CubedSphereLowRankAdvection(24, eps=1e-12)
    q0 = torch.as_tensor(ic.cosine_bell(m.grid.centers(), radius=m.grid.radius))
    F, D = m.to_factored(q0), q0.clone()
    for _ in range(8):
        F, D = m.step(F, m.dt_max), m.dense_step(D, m.dt_max)
    R = m.to_dense(F)
    assert float((R - D).norm() / D.norm()) < 1e-9
    assert abs(m.mass(R) / m.mass(q0) - 1.0) < 1e-12
    assert max(f.rank for f in F) < 24


def test_factored_tc1_against_fv_solver_cpu():
    """One day of TC1 at C32: the factored central scheme (rank <= 12 per
    panel) against the exact rotated bell and the FV solver (PLR, MC limiter,
    torch path) on the same grid and dt.  Measured: L2 0.129 (factored), 0.063
    (FV); the central scheme is the more dispersive, so the gate is 2.5x."""
    from stsphere.engine import Engine
    from stsphere.models import tt
    from stsphere.models import initial_conditions as ic
    from stsphere.models.advection import Advection
    from stsphere.parallel.layout import TileLayout
    N = 32
    m = tt.CubedSphereLowRankAdvection(N, eps=1e-8)
    g = m.grid
    fv = Engine(Advection(limiter=2), TileLayout(N, 1, 1, ng=2), grid=g, backend="torch")
    steps = int(round(86400.0 / fv.dt))
    F = m.to_factored(torch.as_tensor(ic.cosine_bell(g.centers(), radius=g.radius)))
    for _ in range(steps):
        F = m.step(F, fv.dt)
    fv.step(steps)
    ex = torch.as_tensor(ic.cosine_bell_exact(g.centers(), steps * fv.dt, radius=g.radius))
    A = torch.as_tensor(g.areas())
    l2 = lambda q: float(torch.sqrt(((q - ex) ** 2 * A).sum() / (ex ** 2 * A).sum()))
    e_tt = l2(m.to_dense(F))
    e_fv = l2(torch.as_tensor(fv.global_field(0)).reshape(6, N, N))
    assert max(f.rank for f in F) <= 16
    assert e_tt < 0.2 and e_tt < 2.5 * e_fv


def test_lowrank_shallow_water_matches_dense_and_the_dispersion_relation():
    """Factored linearised rotating SWE (PDF s.3): equal to the dense operator
    to 1e-10 after 60 SSP-RK3 steps of a two-mode state, mass conserved, the
    standing inertia-gravity mode at the semi-discrete frequency."""
    import math
    sw = tt.LowRankShallowWater(64, g=1.0, H=1.0, f=2.0, eps=1e-13)
    W, omega, _ = sw.gravity_wave(1, 2, amp=0.1)
    W2, _, _ = sw.gravity_wave(3, 1, amp=0.05)
    W = W + W2
    W[1] += 0.02 * torch.outer(torch.ones(64, dtype=torch.float64), torch.sin(2 * math.pi * torch.arange(64) / 64))
    F = sw.to_factored(W)
    D = W.clone()
    dt = 0.5 * sw.dt_max
    m0 = float(D[0].sum())
    for _ in range(60):
        F, D = sw.step(F, dt), sw.dense_step(D, dt)
    R = sw.to_dense(F)
    assert float((R - D).norm() / D.norm()) < 1e-10
    assert abs(float(R[0].sum()) - m0) < 1e-12 * abs(D[0]).sum()
    assert max(f.rank for f in F) <= 8
    # one mode against its semi-discrete solution h0 (f^2 + gH k'^2 cos wt) / w^2
    sw1 = tt.LowRankShallowWater(64, g=1.0, H=1.0, f=2.0, eps=1e-13)
    W1, om, (kx, ky) = sw1.gravity_wave(1, 2, amp=0.1)
    F1 = sw1.to_factored(W1)
    n = 200
    dt1 = 0.25 * sw1.dt_max
    for _ in range(n):
        F1 = sw1.step(F1, dt1)
    t = n * dt1
    gk2 = sw1.g * sw1.H * (kx * kx + ky * ky)
    want = W1[0] * (sw1.f ** 2 + gk2 * math.cos(om * t)) / om ** 2
    got = sw1.to_dense(F1)[0]
    assert float((got - want).norm() / W1[0].norm()) < 1e-5
    assert F1[0].rank == 1


@pytest.mark.parametrize("N", [12, 20])
def test_cube_lowrank_shallow_water_matches_dense_six_panel_operator(N):
    """Six-panel factored linear SWE (true sphere metric, Cartesian velocity
    exchanged as three scalars across panel edges, PDF s.18) against the
    N x N six-panel reference of the same discrete operator: 1e-10 after four
    SSP-RK3 steps of a gravity-wave hill that crosses panel edges; mass
    sum(A h) conserved to round-off in both; the velocity stays tangent."""
    sw = tt.CubedSphereLowRankShallowWater(N, eps=1e-13)
    W = sw.gaussian_hill()
    F = sw.to_factored(W)
    Wd = W.clone()
    dt = sw.dt_max
    for _ in range(4):
        F = sw.step(F, dt)
        Wd = sw.dense_step(Wd, dt)
    D = sw.to_dense(F)
    assert float((D - Wd).abs().amax() / Wd.abs().amax()) < 1e-10
    m0 = sw.mass(W)
    assert abs(sw.mass(Wd) - m0) < 1e-12 * abs(m0)
    assert abs(sw.mass(D) - m0) < 1e-10 * abs(m0)
    vr = (Wd[1:] * sw.r.permute(3, 0, 1, 2)).sum(0)
    assert float(vr.abs().max()) < 1e-12 * float(Wd[1:].abs().max())
    # the hill moved: gravity waves reached the neighbouring cells, velocities grew
    assert float(Wd[1:].abs().max()) > 0.0
    if N >= 20:                  # factored storage below dense (C12 saturates at rank N)
        assert max(f.rank for Fq in F for f in Fq) < N


def test_cube_lowrank_shallow_water_curvature_sum_kills_constant_gradient():
    """A constant height has no gradient on the sphere (the Gauss sum minus the
    curvature sum S) and a resting constant layer stays at rest."""
    sw = tt.CubedSphereLowRankShallowWater(12)
    W = torch.zeros((4, 6, 12, 12), dtype=torch.float64)
    W[0] = 5.0
    R = sw.dense_rhs(W)
    assert float(R.abs().max()) < 1e-12
    F = sw.to_factored(W)
    Rf = sw.to_dense(sw.rhs(F))
    assert float(Rf.abs().max()) < 1e-9


def test_cube_lowrank_shallow_water_chunked_rounding_cpu(monkeypatch):
    """The hip backend's chunk-by-chunk rounding of wide products
    (``_round_native``: <= min(ROUND_CAP, N / 2) columns per native call, the
    running result carried into the next chunk), with the native call replaced
    by the QR + SVD rounding of the same columns: still the dense operator to
    1e-10."""
    from stsphere.ops import tt_ops

    def fake(A, B, eps, max_rank=None):
        assert A.shape[1] <= min(tt.ROUND_CAP, A.shape[0] // 2, B.shape[0] // 2)
        f = tt.recompress(A, B, eps, max_rank)
        return f.A, f.B

    monkeypatch.setattr(tt_ops, "recompress", fake)
    N = 40
    sw = tt.CubedSphereLowRankShallowWater(N, eps=1e-13)
    sw.backend = "hip"
    W = sw.gaussian_hill()
    F = sw.to_factored(W)
    Wd = W.clone()
    for _ in range(2):
        F = sw.step(F, sw.dt_max)
        Wd = sw.dense_step(Wd, sw.dt_max)
    D = sw.to_dense(F)
    assert float((D - Wd).abs().amax() / Wd.abs().amax()) < 1e-10
    st = sw.stats
    assert st["native"] > st["recompressions"] - st["library"] > 0
