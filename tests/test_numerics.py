"""Numerics of the PyTorch reference path (the oracle the HIP kernels are tested against)."""
import math

import numpy as np
import pytest
import torch

from stsphere.engine import Engine
from stsphere.models.advection import Advection
from stsphere.models.diffusion import Diffusion
from stsphere.models.geometry import DAY, CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.parallel.layout import TileLayout


def _l2(a, b, A):
    return math.sqrt(((a - b) ** 2 * A).sum() / ((b ** 2) * A).sum())


@pytest.mark.parametrize("phys", [lambda: ShallowWater("tc5"), lambda: Advection(), lambda: Diffusion()])
def test_mass_conserved_to_roundoff(phys):
    p = phys()
    e = Engine(p, TileLayout(12, 2, 1, ng=2), integrator="ssprk3")
    m0 = e.diagnostics()["mass"]
    e.step(20)
    assert abs(e.diagnostics()["mass"] / m0 - 1) < 1e-13


def test_swe_tc2_second_order_convergence():
    errs = []
    for N in (12, 24):
        g = CubedSphereGrid(N)
        e = Engine(ShallowWater("tc2"), TileLayout(N, 1, 1, ng=2), grid=g)
        h0 = e.global_field(0)
        days = 1.0
        n = int(math.ceil(days * DAY / e.dt))
        e.dt = days * DAY / n
        e.step(n)
        errs.append(_l2(e.global_field(0), h0, g.areas()))
    order = math.log2(errs[0] / errs[1])
    assert errs[1] < 2e-3 and order > 1.5, (errs, order)


def test_lake_at_rest_is_steady():
    e = Engine(ShallowWater("rest"), TileLayout(8, 1, 1, ng=2))
    q0 = e.tiles_view().clone()
    e.step(10)
    assert (e.tiles_view() - q0).abs().max() < 1e-9 * 1000


def test_tc1_bell_moves_east_across_panel_edge():
    g = CubedSphereGrid(16)
    e = Engine(Advection(), TileLayout(16, 1, 1, ng=2), grid=g)
    q = e.global_field(0)
    assert q[3].max() > 0.9 * q.max()          # starts on face 3 (270E, PDF s.13)
    n = int(math.ceil(3 * DAY / e.dt))
    e.dt = 3 * DAY / n
    e.step(n)                                     # quarter revolution -> face 4 (0E), PDF s.18
    q = e.global_field(0)
    assert q[4].sum() > 5 * q[3].sum()


def test_diffusion_decays_extrema_monotone():
    e = Engine(Diffusion(), TileLayout(16, 1, 1, ng=1), integrator="rk4")
    q0 = e.global_field(0)
    e.step(30)
    q = e.global_field(0)
    assert q.max() < q0.max() and q.min() >= q0.min() - 1e-9


@pytest.mark.parametrize("integ", ["euler", "ssprk2", "ssprk3", "rk4"])
def test_integrators_run_and_agree(integ):
    g = CubedSphereGrid(8)
    e = Engine(ShallowWater("tc2"), TileLayout(8, 1, 1, ng=2), grid=g, integrator=integ)
    h0 = e.global_field(0)
    e.dt = e.dt / 4
    e.step(4)
    assert _l2(e.global_field(0), h0, g.areas()) < 3e-3   # C8: spatial error ~1.7e-3 dominates


def test_ppm_needs_three_ghost_layers():
    p = ShallowWater("tc5", limiter=4)
    assert p.halo == 3 and ShallowWater("tc5").halo == 2
    with pytest.raises(ValueError):
        Engine(p, TileLayout(12, 1, 1, ng=2))


@pytest.mark.parametrize("phys", [lambda: ShallowWater("tc5", limiter=4), lambda: Advection(limiter=4)])
def test_ppm_conserves_mass(phys):
    e = Engine(phys(), TileLayout(12, 2, 1, ng=3))
    m0 = e.diagnostics()["mass"]
    e.step(20)
    assert abs(e.diagnostics()["mass"] / m0 - 1) < 1e-13
    assert bool(torch.isfinite(e.tiles_view()).all())


def _tc2_error(N, lim):
    g = CubedSphereGrid(N)
    e = Engine(ShallowWater("tc2", limiter=lim), TileLayout(N, 1, 1, ng=3 if lim == 4 else 2), grid=g)
    h0 = e.global_field(0)
    m0 = e.diagnostics()["mass"]
    n = int(math.ceil(DAY / e.dt))
    e.dt = DAY / n
    e.step(n)
    assert abs(e.diagnostics()["mass"] / m0 - 1) < 1e-13      # single-valued panel-edge fluxes
    return _l2(e.global_field(0), h0, g.areas())


def test_panel_edge_reconstruction_keeps_second_order_tc2():
    """Steady geostrophic flow (TC2), one day, C24 -> C48.  With ghost values
    interpolated along the neighbouring panel's grid lines (Putman & Lin 2007,
    PDF s.14) and the neighbour's edge state reconstructed in its own frame,
    MC-PLR and PPM both converge at second order across the cube edges, and
    PPM is the more accurate.  Measured (CPU fp64): MC 4.63e-4 -> 7.74e-5
    (order 2.58), PPM 2.56e-4 -> 6.82e-5 (1.91); with the index-space ghost
    copy of round 1 it was MC 1.34e-3 -> 3.84e-4 (1.81), PPM 1.20e-3 -> 4.39e-4
    (1.45, worse than PLR at C48)."""
    mc = [_tc2_error(N, 2) for N in (24, 48)]
    ppm = [_tc2_error(N, 4) for N in (24, 48)]
    assert math.log2(mc[0] / mc[1]) >= 1.8, mc
    assert math.log2(ppm[0] / ppm[1]) >= 1.8, ppm
    assert ppm[1] <= mc[1], (ppm, mc)
    assert mc[1] < 1e-4 and ppm[1] < 1e-4


def test_panel_edges_are_decomposition_independent():
    """SURVEY.md 7.4 item 6 / VERDICT r3 item 7: the panel-edge ghost pair is
    chosen on the whole panel edge and the strip cells beyond a tile end come
    from the diagonal tile as carried corner ghosts, so the TC2 state after one
    day is the same with 1, 2 and 4 tiles per edge (to 1e-12 relative; the
    torch path gives it bitwise), and mass is conserved to roundoff."""
    states = []
    for t in (1, 2, 4):
        g = CubedSphereGrid(24)
        e = Engine(ShallowWater("tc2"), TileLayout(24, t, 1, ng=2), grid=g)
        m0 = e.diagnostics()["mass"]
        n = int(math.ceil(DAY / e.dt))
        e.dt = DAY / n
        e.step(n)
        assert abs(e.diagnostics()["mass"] / m0 - 1) < 1e-13
        states.append(np.stack([e.global_field(f) for f in range(e.physics.F)]))
    for s in states[1:]:
        assert np.abs(s - states[0]).max() <= 1e-12 * np.abs(states[0]).max()


@pytest.mark.parametrize("mk", [lambda: ShallowWater("tc5", limiter=4), lambda: Advection(limiter=4)])
def test_ppm_panel_edges_are_decomposition_independent(mk):
    """PPM reads two interpolated ghost layers, whose pairs reach up to two
    cells beyond a tile end (t = 4 places tile boundaries where the pull is
    largest): 1, 2 and 4 tiles per edge agree bitwise."""
    out = []
    for t in (1, 2, 4):
        e = Engine(mk(), TileLayout(24, t, 1, ng=3), grid=CubedSphereGrid(24))
        e.step(5)
        out.append(np.stack([e.global_field(f) for f in range(e.physics.F)]))
    for s in out[1:]:
        assert np.array_equal(s, out[0])


def test_decomposition_independent_across_ranks():
    """Remote carried corners: a 4-rank in-process run of C24 t = 2 equals
    one rank holding every tile, bitwise."""
    from stsphere.engine import VirtualCluster
    g = CubedSphereGrid(24)
    one = Engine(ShallowWater("tc5"), TileLayout(24, 2, 1, ng=2), grid=g)
    vc = VirtualCluster(lambda: ShallowWater("tc5"), TileLayout(24, 2, 4, ng=2), grid=g, dt=one.dt)
    one.step(4)
    vc.step(4)
    assert np.array_equal(vc.global_field(0), one.global_field(0))


def test_panel_edge_tables_follow_the_neighbours_grid_lines():
    """The interpolation target of ghost layer k on panel-edge strips is
    beta' = atan(tan(beta) / tan(pi/4 + delta_k)): at the edge middle it stays
    on the row, toward the cube corners it is pulled inward by up to k + 1/2
    cells, symmetrically; the pair is chosen on the whole panel edge (the same
    global pair for every decomposition), leaving the tile by at most k + 1
    cells, into the carried corner ghosts."""
    from stsphere.models.base import panel_edge_target, panel_edge_tables
    N = 24
    J = np.arange(N)
    for k in range(3):
        u = panel_edge_target(N, J, k)
        assert np.allclose(u + u[::-1], N - 1)                  # mirror symmetric
        assert np.all(np.abs(u - J) <= k + 0.5 + 1e-12)
        assert np.all(np.sign(u - J) == -np.sign(J - (N - 1) / 2))
    b1, t1 = panel_edge_tables(N, TileLayout(N, 1, 1, ng=3), [0], 3)
    assert b1.min() >= 0 and b1.max() <= N - 2
    for t in (2, 4):
        L = TileLayout(N, t, 1, ng=3)
        b, tt = panel_edge_tables(N, L, L.plan(0).tiles, 3)
        n = L.n
        for k in range(3):
            assert b[:, :, k].min() >= -(k + 1) and b[:, :, k].max() + 1 <= n + k
        for li, tid in enumerate(L.plan(0).tiles):
            f, I0, J0 = L.tile_origin(tid)
            for s in range(4):
                o = J0 if s < 2 else I0
                assert np.array_equal(b[li, s] + o, b1[0, s][:, o:o + n])
                assert np.array_equal(tt[li, s], t1[0, s][:, o:o + n])


def test_ppm_advection_keeps_the_peak():
    """PPM is markedly less diffusive than PLR on the cosine bell (peak after
    40 steps at C16: ~726 vs ~595 of 897), with only a small undershoot
    (the MOL form is not strictly TVD)."""
    peaks = {}
    for lim, ng in ((2, 2), (4, 3)):
        e = Engine(Advection(limiter=lim), TileLayout(16, 1, 1, ng=ng))
        q0max = float(e.tiles_view().max())
        e.step(40)
        q = e.tiles_view()
        peaks[lim] = float(q.max())
        assert float(q.max()) <= q0max * (1 + 1e-12)
        assert float(q.min()) > -0.02 * q0max
    assert peaks[4] > 1.1 * peaks[2], peaks


@pytest.mark.parametrize("alpha", [0.0, math.pi / 4])
def test_tc1_one_revolution_williamson_norms(alpha):
    """Williamson TC1 after one full revolution (12 days), PLR + MC, SSP-RK3.
    Measured (CPU, fp64, panel-edge interpolation): alpha=pi/4: l2 0.478 (C24)
    -> 0.167 (C48) -> 0.0588 (C96), orders 1.52 / 1.50.  The MC limiter clips
    the bell's peak, which bounds PLR's order here (unlimited central PLR:
    1.17 / 1.69 with larger errors); PPM: see the next test."""
    from stsphere.models.errors import convergence_order, williamson_norms
    errs = []
    for N in (24, 48):
        g = CubedSphereGrid(N)
        ph = Advection(alpha=alpha)
        e = Engine(ph, TileLayout(N, 1, 1, ng=2), grid=g)
        n = int(math.ceil(12 * DAY / e.dt))
        e.dt = 12 * DAY / n
        e.step(n)
        nr = williamson_norms(e.global_field(0), ph.exact(g, e.time), g.areas())
        assert nr["linf"] < 0.6 and nr["l1"] < 0.7
        errs.append(nr["l2"])
    assert errs[1] < 0.2, errs
    # measured orders C24 -> C48: 1.30 (alpha = 0, the bell runs along the
    # panel edges' equator), 1.52 (alpha = pi/4)
    assert convergence_order(errs, (24, 48)) > (1.2 if alpha == 0.0 else 1.42), errs


def test_tc1_ppm_converges_c48_c96():
    """TC1 (alpha = pi/4), one revolution, PPM faces with the panel-edge
    treatment: l2 0.0762 (C48) -> 0.0214 (C96), order 1.83 (CPU fp64)."""
    from stsphere.models.errors import convergence_order, williamson_norms
    errs = []
    for N in (48, 96):
        g = CubedSphereGrid(N)
        ph = Advection(alpha=math.pi / 4, limiter=4)
        e = Engine(ph, TileLayout(N, 1, 1, ng=3), grid=g)
        n = int(math.ceil(12 * DAY / e.dt))
        e.dt = 12 * DAY / n
        e.step(n)
        errs.append(williamson_norms(e.global_field(0), ph.exact(g, e.time), g.areas())["l2"])
    assert convergence_order(errs, (48, 96)) >= 1.73, errs
    assert errs[1] < 0.025, errs


def _restrict(h, A, r):
    """Conservative restriction of a [6, N, N] cell-average field by r x r."""
    M = h.shape[1] // r
    hA = (h * A).reshape(6, M, r, M, r).sum((2, 4))
    AA = A.reshape(6, M, r, M, r).sum((2, 4))
    return hA / AA, AA


def test_tc5_self_convergence_second_order():
    """Williamson TC5 (flow over the mountain), 3 hours, MC-PLR + SSP-RK3 at
    the bench's CFL: h of C24 / C48 / C96 against the C192 solution restricted
    conservatively to each grid.  The reference holds no TC5 numbers (parity
    unpinned), so self-convergence is the pin: order >= 1.8 from C24 to C96
    and on the finest pair (C24 is pre-asymptotic: the mountain spans ~4
    cells).  Measured (CPU fp64): 1.39e-3 (C24), 4.13e-4 (C48), 1.02e-4
    (C96): orders 1.75, 2.01, overall 1.88."""
    T = 3 * 3600.0
    sol = {}
    for N in (24, 48, 96, 192):
        g = CubedSphereGrid(N)
        e = Engine(ShallowWater("tc5"), TileLayout(N, 1, 1, ng=2), grid=g)
        n = int(math.ceil(T / e.dt))
        e.dt = T / n
        e.step(n)
        sol[N] = (e.global_field(0), g.areas())
    href, Aref = sol[192]
    errs = []
    for N in (24, 48, 96):
        hr, _ = _restrict(href, Aref, 192 // N)
        h, A = sol[N]
        errs.append(_l2(h, hr, A))
    o1, o2 = math.log2(errs[0] / errs[1]), math.log2(errs[1] / errs[2])
    assert o2 >= 1.9 and o1 >= 1.65 and (o1 + o2) / 2 >= 1.8, (errs, o1, o2)
    assert errs[2] < 1.5e-4, errs


def test_tc6_energy_dissipation_converges():
    """Williamson TC6 (Rossby-Haurwitz wave 4), one day: total energy
    (kinetic + potential, models/swe.py) only decays (Rusanov + limiter
    dissipation), by < 5e-4 at C48, and the loss shrinks at >= 2.5 orders
    per refinement; mass to roundoff.  Measured (CPU fp64): -2.69e-3 (C24),
    -3.42e-4 (C48), order 2.97."""
    drift = []
    for N in (24, 48):
        g = CubedSphereGrid(N)
        e = Engine(ShallowWater("tc6"), TileLayout(N, 1, 1, ng=2), grid=g)
        d0 = e.diagnostics()
        n = int(math.ceil(DAY / e.dt))
        e.dt = DAY / n
        e.step(n)
        d1 = e.diagnostics()
        assert abs(d1["mass"] / d0["mass"] - 1) < 1e-12
        drift.append(d1["energy"] / d0["energy"] - 1)
    assert drift[0] < 0 and drift[1] < 0, drift
    assert abs(drift[1]) < 5e-4, drift
    assert math.log2(drift[0] / drift[1]) >= 2.5, drift


def test_williamson_norms_definition():
    from stsphere.models.errors import convergence_order, williamson_norms
    t = np.array([1.0, 2.0, -2.0])
    a = np.array([1.0, 1.0, 2.0])
    nr = williamson_norms(t + np.array([0.1, 0.0, -0.2]), t, a)
    assert math.isclose(nr["l1"], (0.1 + 0.4) / 7.0)
    assert math.isclose(nr["l2"], math.sqrt((0.01 + 0.08) / 13.0))
    assert math.isclose(nr["linf"], 0.2 / 2.0)
    assert math.isclose(convergence_order([4.0, 1.0], [10, 20]), 2.0)


@pytest.mark.parametrize("mk", [lambda: ShallowWater("tc5"), lambda: ShallowWater("tc5", limiter=4),
                                lambda: Advection(), lambda: Advection(limiter=4), lambda: Diffusion()])
@pytest.mark.parametrize("t", [1, 2])
def test_no_stencil_reads_a_corner_ghost(mk, t):
    """Tile-corner ghost blocks (cube corners included) are never written; with
    every one of them NaN the state stays finite and bitwise equal to the
    zero-corner run (the zeros were an unguarded assumption)."""
    from stsphere.engine import Engine
    from stsphere.parallel.layout import TileLayout
    N = 12
    g = CubedSphereGrid(N)
    phys = mk()
    ng = 3 if getattr(phys, "limiter", 0) == 4 else 2
    a = Engine(mk(), TileLayout(N, t, 1, ng=ng), grid=g)
    b = Engine(mk(), TileLayout(N, t, 1, ng=ng), grid=g, dt=a.dt)
    b.poison_corners()
    assert b.corner_slots().numel() == b.plan.T * 4 * ng * ng - int(b.plan.corner_carried.sum())
    assert (t == 1) == (int(b.plan.corner_carried.sum()) == 0)
    a.step(3)
    b.step(3)
    assert torch.isfinite(b.tiles_view()).all()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert torch.isnan(b.state[:, b.corner_slots()]).all()
