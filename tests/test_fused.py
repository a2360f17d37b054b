"""Fused SSP-RK3 step (temporal blocking, ops/fused.py + ops/csrc/fused_step.hip)
against the stage-by-stage PyTorch oracle.

CPU: the PyTorch rendering of the fused algorithm (FusedTorch, the same host
tables and phases as the kernel) reproduces Engine.step to rounding on grids
whose windows cross one panel edge, two panel edges, and cube corners.
GPU: the gfx950 kernel against the fp64 oracle (1e-11), fp32 (1e-4), graph
replay vs eager (bitwise), and a corner-poison check."""
import numpy as np
import pytest
import torch

from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.ops.fused import FusedPlan, FusedTorch, fused_supported, region
from stsphere.parallel.layout import TileLayout


def _relerr(a_eng, b_eng):
    a = a_eng.tiles_view().reshape(4, -1).double()
    b = b_eng.tiles_view().reshape(4, -1).double()
    return ((a - b).abs().amax(1) / a.abs().amax(1)).max().item()


@pytest.mark.parametrize("N,t,B,case,lim", [
    (16, 1, 8, "tc5", 2),     # one panel edge per window side, cube corners
    (24, 2, 4, "tc5", 2),     # two tiles per panel edge, tile-clipped interpolation
    (12, 1, 4, "tc2", 1),     # windows that cross both opposite panel edges
    (24, 1, 8, "tc6", 3),
    (36, 2, 18, "tc5", 2),    # the B = 18 kernel shape (C180 / C720 tiles)
])
def test_fused_torch_matches_stage_oracle(N, t, B, case, lim):
    grid = CubedSphereGrid(N)
    L = TileLayout(N, t, 1, ng=2)
    ref = Engine(ShallowWater(case, limiter=lim), L, grid=grid)
    fe = Engine(ShallowWater(case, limiter=lim), L, grid=grid, dt=ref.dt)
    ft = FusedTorch(fe, FusedPlan(L, 0, grid, B=B, ns=3))
    for _ in range(2):
        ref.step(1)
        ft.step()
    assert _relerr(ref, fe) < 1e-12
    assert fe.step_count == 2


@pytest.mark.parametrize("B", [6, 8, 12, 16, 18, 20])
def test_pass_schedule_covers_every_pass_once(B):
    """Every face pass of every stage runs on exactly one wave (the kernel's
    per-wave masks), the corner wave and the ghost waves exist in the thread
    count, and the balanced schedule's busiest SIMD group never carries more
    than round 4's placement ("legacy")."""
    from stsphere.ops.fused import fused_threads, pass_masks, pass_schedule, stage_face_counts
    nw = fused_threads(B) // 64
    ncor = np.array([0, 0, 7, 30])
    edge = np.array([False, True, True, True])
    counts = stage_face_counts(B)
    for w in ("8:1", "legacy"):
        sc = pass_schedule(B, ncor, edge, 88, weights=w)
        m = pass_masks(B, sc)
        assert m.shape == (4, 3, 17) and int(sc.max()) < nw
        for s_, cnt in enumerate(counts):
            npass = -(-cnt // 64)
            assert npass <= 32
            allp = np.bitwise_or.reduce(m[:, s_, :16], axis=1)
            assert (allp == np.uint32((1 << npass) - 1)).all()
            for b in range(4):       # no pass twice
                bits = sum(bin(int(x)).count("1") for x in m[b, s_, :16])
                assert bits == npass

    def group_load(sc, b, s_, wc=8, wg=1):
        cw = 1 if ncor[b] else 0
        gw = 2 if edge[b] else 0
        wl = [0] * nw
        if cw:
            wl[0] += wc
        for w_ in range(cw, cw + gw):
            wl[w_] += wg
        for p in range(-(-counts[s_] // 64)):
            wl[int(sc[b, s_, p])] += 4
        return max(sum(wl[w_] for w_ in range(g, nw, 4)) for g in range(4))

    new, old = pass_schedule(B, ncor, edge, 88), pass_schedule(B, ncor, edge, 88, weights="legacy")
    for b in range(4):
        for s_ in range(3):
            assert group_load(new, b, s_) <= group_load(old, b, s_)


@pytest.mark.parametrize("N,B", [(48, 16), (48, 6), (36, 6)])
def test_near_pass_masks_flag_every_near_face(N, B):
    """A face pass the host does not flag must hold no face within one line
    of a panel-edge line (those faces read neighbour codes and ghost entries;
    an unflagged one would read the raw window), and interior blocks flag
    nothing.  B = 6: the small rank-share blocks."""
    from stsphere.ops.fused import near_pass_masks, stage_face_coords
    L = TileLayout(N, 1, 1, ng=2)
    P = FusedPlan(L, 0, CubedSphereGrid(N), B=B, ns=3)
    flags = np.array([sum(1 << int(r) for r in np.unique(P.reg[b]) if r >= 0) for b in range(P.nb)])
    nm = near_pass_masks(B, P.org, flags, N)
    coords = stage_face_coords(B)
    W = P.d.W
    for b in range(P.nb):
        X0, Y0 = int(P.org[b, 0]), int(P.org[b, 1])
        if flags[b] == 1:
            assert (nm[b] == 0).all()
            continue
        lines = {0: [k for k in range(W + 1) if ((flags[b] & 2) and abs(k - (-X0)) <= 1)
                     or ((flags[b] & 4) and abs(k - (N - X0)) <= 1)],
                 1: [k for k in range(W + 1) if ((flags[b] & 8) and abs(k - (-Y0)) <= 1)
                     or ((flags[b] & 16) and abs(k - (N - Y0)) <= 1)]}
        for s_, (ax, k, _) in enumerate(coords):
            for t in range(len(k)):
                if int(k[t]) in lines[int(ax[t])]:
                    assert (int(nm[b, s_]) >> (t // 64)) & 1, (b, s_, t)
    assert nm.any()


def test_face_normals_match_region_tables():
    """The per-face normal table of panel-edge blocks is the region line-normal
    table at the face's lower-cell region (the kernel's non-PFN path)."""
    from stsphere.ops.fused import face_normals
    N, B = 32, 16
    L = TileLayout(N, 2, 1, ng=2)
    P = FusedPlan(L, 0, CubedSphereGrid(N), B=B, ns=3)
    flags = np.array([sum(1 << int(r) for r in np.unique(P.reg[b]) if r >= 0) for b in range(P.nb)])
    nf = face_normals(P, flags)
    d = P.d
    rng = np.random.default_rng(0)
    for b in np.nonzero(flags != 1)[0][:6]:
        for j in rng.integers(0, 2 * d.nfx, 40):
            yf = j >= d.nfx
            jj = j - d.nfx if yf else j
            r, c = divmod(int(jj), d.H1 if yf else d.H1 + 1)
            fu, fv = d.L1 + c, d.L1 + r
            k = fv if yf else fu
            lu, lv = (fu, fv - 1) if yf else (fu - 1, fv)
            ra = int(region(P.org[b, 0] + lu, P.org[b, 1] + lv, N))
            ra = max(ra, 0)
            assert np.array_equal(nf[b, :, j], P.nrm[b, int(yf), ra, k, :])
    assert (nf[flags == 1] == 0).all()


def test_fused_plan_invariants():
    N, B = 32, 16
    L = TileLayout(N, 2, 1, ng=2)
    P = FusedPlan(L, 0, CubedSphereGrid(N), B=B, ns=3)
    d = P.d
    assert (d.W, d.R, d.L1, d.H1) == (28, 6, 2, 24)
    W = d.W
    for b in range(P.nb):
        reg = P.reg[b].reshape(W, W)
        X0, Y0 = P.org[b, 0], P.org[b, 1]
        vv, uu = np.mgrid[0:W, 0:W]
        assert (region(X0 + uu, Y0 + vv, N) == reg).all()
        # every needed cell exists and is loaded; stage s needs lie in its square
        assert (P.src[b][P.need[b, 0]] >= 0).all()
        for s in range(1, d.ns + 1):
            lo, hi = d.stage_range(s)
            m = P.need[b, s].reshape(W, W)
            assert not m[:lo].any() and not m[hi:].any() and not m[:, :lo].any() and not m[:, hi:].any()
            assert (P.need[b, s] <= P.need[b, s - 1]).all()
        # ghost entries name two window cells and a weight in [-1, 2]
        k = int(P.gcnt[b])
        assert ((P.gtab[b, :k, 2:] >= 0) & (P.gtab[b, :k, 2:] < W * W)).all()
        assert (np.abs(P.gt[b, :k]) <= 2).all()
    # cube-corner blocks have corner faces
    assert P.ccnt.max() > 0


def test_fused_supported_reasons():
    L = TileLayout(24, 1, 1, ng=2)
    e = Engine(ShallowWater("tc5", limiter=4), TileLayout(24, 1, 1, ng=3))
    assert "PLR" in fused_supported(e)
    e = Engine(ShallowWater("tc5"), L, integrator="rk4")
    assert "SSP-RK3" in fused_supported(e)
    e = Engine(ShallowWater("tc5"), TileLayout(28, 2, 1, ng=2))
    assert "multiple of 6 or 8 or 12 or 16 or 18 or 20" in fused_supported(e)
    assert fused_supported(Engine(ShallowWater("tc5"), TileLayout(24, 2, 1, ng=2))) is None   # B = 12
    assert fused_supported(Engine(ShallowWater("tc5"), TileLayout(36, 2, 1, ng=2))) is None   # B = 18
    assert fused_supported(Engine(ShallowWater("tc5"), TileLayout(40, 2, 1, ng=2))) is None   # B = 20
    e = Engine(ShallowWater("tc5"), TileLayout(32, 2, 1, ng=2))
    assert fused_supported(e) is None


# ---------------------------------------------------------------------------
# GPU: the gfx950 kernel
# ---------------------------------------------------------------------------

def _gpu_pair(N, t, dtype=torch.float64, case="tc5", lim=2):
    grid = CubedSphereGrid(N)
    L = TileLayout(N, t, 1, ng=2)
    ref = Engine(ShallowWater(case, limiter=lim), L, grid=grid, dtype=torch.float64, device="cuda", backend="torch")
    hip = Engine(ShallowWater(case, limiter=lim), L, grid=grid, dtype=dtype, device="cuda", backend="hip", dt=ref.dt)
    return ref, hip


@pytest.mark.gpu
@pytest.mark.parametrize("N,t,case,lim", [(32, 2, "tc5", 2), (48, 1, "tc5", 1), (96, 2, "tc5", 2),
                                          (48, 3, "tc6", 3), (32, 1, "tc2", 0), (36, 2, "tc5", 2),
                                          (54, 1, "tc2", 1), (40, 2, "tc5", 2), (60, 3, "tc6", 2),
                                          (48, 4, "tc5", 2), (72, 3, "tc5", 2)])
def test_fused_kernel_fp64_matches_oracle(N, t, case, lim):
    """Every block size through the residency-aware choice: 6 (36, 2), 8 ((32, 2),
    (48, 1), (48, 3), (32, 1)), 12 ((48, 4), (72, 3)), 16 (96, 2), 18 (54, 1), 20."""
    from stsphere.ops.fused import FusedKernel
    ref, hip = _gpu_pair(N, t, case=case, lim=lim)
    fk = FusedKernel(hip)
    for _ in range(3):
        ref.step(1)
        fk.step(1)
        torch.cuda.synchronize()
        assert _relerr(ref, hip) < 1e-11


@pytest.mark.gpu
@pytest.mark.parametrize("N,t,case,lim", [(36, 1, "tc5", 2), (24, 2, "tc6", 3), (12, 1, "tc2", 1)])
def test_fused_kernel_b6_matches_oracle_and_multi_step(N, t, case, lim):
    """The B = 6 instance (a rank's share of C96 over 8 GPUs: 3 tiles of 48,
    192 blocks): the oracle at 1e-11 over single-step launches, and a
    multi-step launch bitwise equal to single steps."""
    from stsphere.ops.fused import FusedKernel
    ref, hip = _gpu_pair(N, t, case=case, lim=lim)
    fk = FusedKernel(hip, B=6)
    for _ in range(2):
        ref.step(1)
        fk.step(1)
        torch.cuda.synchronize()
        assert _relerr(ref, hip) < 1e-11
    from stsphere.ops.native_runtime import NativeStepper
    _, a = _gpu_pair(N, t, case=case, lim=lim)
    _, b = _gpu_pair(N, t, case=case, lim=lim)
    b.dt = a.dt
    FusedKernel(a, B=6).step(6)
    fb = FusedKernel(b, B=6)
    r = NativeStepper(b, use_graph=True, steps_per_graph=6, fused=fb, steps_per_launch=6)
    r.run(6)
    torch.cuda.synchronize()
    fb.check()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    r.close()


@pytest.mark.gpu
def test_fused_kernel_matches_stage_kernel_and_halos():
    """Fused vs the launch-per-stage kernel over 6 steps; the fused step also
    leaves every same-rank ghost slot current (it pushes like the stage kernel)."""
    from stsphere.ops.fused import FusedKernel
    _, a = _gpu_pair(48, 3)
    _, b = _gpu_pair(48, 3)
    b.dt = a.dt
    fk = FusedKernel(b)
    a.step(6)
    fk.step(6)
    torch.cuda.synchronize()
    assert _relerr(a, b) < 1e-11
    q = b.pool[0]
    assert torch.equal(q[:, b.halo_dst], q[:, b.halo_src])


@pytest.mark.gpu
def test_fused_kernel_fp32_close_to_fp64_oracle():
    from stsphere.ops.fused import FusedKernel
    ref, hip = _gpu_pair(48, 3, dtype=torch.float32)
    fk = FusedKernel(hip)
    ref.step(3)
    fk.step(3)
    torch.cuda.synchronize()
    assert _relerr(ref, hip) < 1e-4


@pytest.mark.gpu
def test_fused_kernel_never_reads_corner_ghosts():
    """Corner ghost blocks of the padded storage (no single source at a cube
    corner) are poisoned with NaN: the fused window gathers every cell from its
    source, so the state stays finite and equal to the unpoisoned run."""
    from stsphere.ops.fused import FusedKernel
    _, a = _gpu_pair(32, 2)
    _, b = _gpu_pair(32, 2)
    b.dt = a.dt
    b.poison_corners()
    fa, fb = FusedKernel(a), FusedKernel(b)
    fa.step(3)
    fb.step(3)
    torch.cuda.synchronize()
    assert torch.isfinite(b.tiles_view()).all()
    assert torch.equal(a.tiles_view(), b.tiles_view())


@pytest.mark.gpu
@pytest.mark.parametrize("nsteps", [6, 5])
def test_fused_native_graph_equals_eager(nsteps):
    """NativeStepper(fused=...) replays hipGraphs of fused launches (period 2,
    odd counts end with one eager fused step): bitwise equal to eager steps."""
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.native_runtime import NativeStepper
    _, a = _gpu_pair(32, 2)
    _, b = _gpu_pair(32, 2)
    b.dt = a.dt
    FusedKernel(a).step(nsteps)
    r = NativeStepper(b, use_graph=True, steps_per_graph=4, fused=FusedKernel(b))
    r.run(nsteps)
    torch.cuda.synchronize()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert b.step_count == nsteps
    assert r.stats["graph_steps"] == (nsteps // 2) * 2
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("N,t,spl,nsteps", [(32, 2, 4, 9), (96, 2, 10, 20), (48, 1, 6, 13)])
def test_fused_multi_step_launch_equals_single_steps(N, t, spl, nsteps):
    """Several steps inside one launch (in-kernel producer waits, write-through
    hand-off, ping-pong buffers): bitwise equal to one launch per step,
    through NativeStepper graphs (remainders: an even multi-step launch plus
    one single step), including the ghost slots pushed after the last step."""
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.native_runtime import NativeStepper
    _, a = _gpu_pair(N, t)
    _, b = _gpu_pair(N, t)
    b.dt = a.dt
    FusedKernel(a).step(nsteps)
    fk = FusedKernel(b)
    r = NativeStepper(b, use_graph=True, steps_per_graph=2 * spl, fused=fk, steps_per_launch=spl)
    r.run(nsteps)
    torch.cuda.synchronize()
    fk.check()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert torch.equal(a.pool[0], b.pool[0])
    assert b.step_count == nsteps
    assert r.stats["graph_steps"] == (nsteps // spl) * spl
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_fused_back_to_back_multi_step_launches(dtype):
    """Three back-to-back 8-step launches (the per-block step counters keep
    counting across launches, the ping-pong buffers are reused) equal 24
    single-step launches bit for bit, in fp64 and fp32, and no wait timed out."""
    from stsphere.ops.fused import FusedKernel
    _, a = _gpu_pair(96, 2, dtype=dtype)
    _, b = _gpu_pair(96, 2, dtype=dtype)
    b.dt = a.dt
    FusedKernel(a).step(24)
    fk = FusedKernel(b)
    for _ in range(3):
        fk.launch(0, nsteps=8)
    torch.cuda.synchronize()
    fk.check()
    assert int(fk.tens["epoch"].min()) == int(fk.tens["epoch"].max()) == 24
    assert torch.equal(a.pool[0], b.pool[0])


@pytest.mark.gpu
def test_fused_multi_step_after_odd_single_steps():
    """A multi-step launch after an odd number of eager step() calls (which
    swap the engine's buffers) starts from the current state: its descriptor
    follows the engine's buffer order."""
    from stsphere.ops.fused import FusedKernel
    _, a = _gpu_pair(32, 2)
    _, b = _gpu_pair(32, 2)
    b.dt = a.dt
    FusedKernel(a).step(7)
    fk = FusedKernel(b)
    fk.launch(0, nsteps=2)          # builds (and caches) the 2-step descriptor
    fk.step(1)                      # odd: pool order swapped
    fk.launch(0, nsteps=4)
    torch.cuda.synchronize()
    fk.check()
    assert torch.equal(a.pool[0], b.pool[0])


@pytest.mark.parametrize("N,t,R", [(32, 2, 2), (32, 2, 8), (48, 1, 6), (32, 2, 3)])
def test_fused_exchange_ranks_equal_one_rank(N, t, R):
    """Several ranks (FusedExchangePlan): each rank's window reads its remote
    cells from a receive buffer filled in the slot order of the plan; every
    rank steps with the PyTorch rendering of the kernel.  The assembled state
    equals the one-rank fused step bit for bit, and every producer entry
    delivers exactly the cell its consumer slot names."""
    from stsphere.engine import assemble_global
    from stsphere.ops.fused import FusedExchangePlan, XG_SLOT_BITS
    grid = CubedSphereGrid(N)
    L1 = TileLayout(N, t, 1, ng=2)
    one = Engine(ShallowWater("tc5"), L1, grid=grid)
    f1 = FusedTorch(one, FusedPlan(L1, 0, grid, B=16))
    L = TileLayout(N, t, R, ng=2)
    X = FusedExchangePlan(L, grid, 16)
    engs = [Engine(ShallowWater("tc5"), L, r, grid=grid, dt=one.dt) for r in range(R)]
    fts = [FusedTorch(engs[r], X.plans[r], remote_cells=X.need_remote[r]) for r in range(R)]
    for r in range(R):        # producer codes deliver the consumer's slot cells
        xpush, psrc, pcode = X.producer(r)
        for s_, c in zip(psrc.tolist(), pcode.tolist()):
            p, slot = c >> XG_SLOT_BITS, c & ((1 << XG_SLOT_BITS) - 1)
            assert int(L.local_flat(X.need_remote[p][slot:slot + 1])[0]) == s_
    for _ in range(2):
        f1.step()
        states = [e.pool[0] for e in engs]
        recvs = []
        for r in range(R):
            g = X.need_remote[r]
            tid, _, _ = L.locate(g)
            own = np.asarray(L.owner)[tid]
            off = L.local_flat(g)
            rv = torch.stack([states[int(o)][:, int(k)] for o, k in zip(own, off)]) if len(g) else None
            recvs.append(rv)
        for r in range(R):
            fts[r].step(recvs[r])
    a = np.stack([one.global_field(f) for f in range(4)])
    b = np.stack([assemble_global(L, {e.rank: e.tiles_view()[f].numpy() for e in engs}) for f in range(4)])
    assert np.array_equal(a, b)


def test_kernel_tables_cpu():
    """Host tables the gfx950 kernel reads, checked on CPU: the neighbour
    codes name every ghost entry of the block exactly where the PyTorch
    rendering substitutes, cells beyond a cube corner are -3; the cell record's
    curvature sum S reproduces the oracle's curvature balance (models/swe.py)."""
    from stsphere.ops.fused import global_cell_records, neighbour_codes
    N = 32
    L = TileLayout(N, 2, 1, ng=2)
    grid = CubedSphereGrid(N)
    e = Engine(ShallowWater("tc5"), L, grid=grid)
    P = FusedPlan(L, 0, grid, B=16)
    ft = FusedTorch(e, P)
    codes = neighbour_codes(P)
    W = P.d.W
    c = np.stack([((codes >> np.uint64(16 * k)) & np.uint64(0xFFFF)).astype(np.int64) for k in range(4)], 1)
    c = np.where(c >= 0x8000, c - 0x10000, c).reshape(P.nb, 4, W, W)
    sub = ft.sub.numpy()
    reg = P.reg.reshape(P.nb, W, W)
    valid = reg >= 0
    assert (c[np.broadcast_to(~valid[:, None], c.shape)] == -3).all()
    ok = np.broadcast_to(valid[:, None], c.shape)
    assert np.array_equal(np.where(ok, c, -1), np.where(ok, sub, -1))
    # cube-corner faces resolved on the host: every stencil index is a window
    # cell (interpolation pairs of ghost entries included), the plain ones are
    # the cell itself (across) or its window neighbour (inward)
    from stsphere.ops.fused import corner_tables
    WS = W + 1
    ld = lambda s_: (s_ // W) * WS + s_ % W
    gpair = np.stack([ld(P.gtab[..., 2]), ld(P.gtab[..., 3])], -1)
    ct, cg = corner_tables(P, codes, gpair)
    assert P.ccnt.max() > 0
    for b in range(P.nb):
        for j in range(int(P.ccnt[b])):
            r = ct[b, j]
            assert ((r[:10] >= 0) & (r[:10] < W * WS)).all()
            assert (r[10], r[11]) == (P.ctab[b, j, 4], P.ctab[b, j, 5])
            for q in range(2):
                ic, a0, a1, n0, n1 = r[5 * q:5 * q + 5]
                if not (r[12] >> (2 * q)) & 1:
                    assert a0 == a1 == ic and cg[b, j, 4 + 2 * q] == 0.0
                if not (r[12] >> (2 * q + 1)) & 1:
                    assert n0 == n1 and abs(int(n0) - int(ic)) in (1, WS)
    rec = global_cell_records(e)
    loc = e.geo.gather_global(rec[:, 7:10].reshape(6, N, N, 3))          # [T,n,n,3]
    sbal = e.tens["sbal"].permute(1, 2, 3, 0).numpy()                    # 0.5 g S / A
    want = 0.5 * e.physics.g * loc / e.geo.area[..., None]
    assert np.allclose(sbal, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())


def _to_global(fr, xi, xj, xn):
    ai, aj = fr & 3, (fr >> 2) & 3
    xi, xj, xn = (-xi if fr & 64 else xi), (-xj if fr & 128 else xj), (-xn if fr & 256 else xn)
    return np.array([xi if ai == c else (xj if aj == c else xn) for c in range(3)])


@pytest.mark.parametrize("N,t,B", [(64, 2, 16), (72, 2, 18)])
def test_kernel_geometry_reconstruction_cpu(N, t, B):
    """The fused kernel's prologue reads panel-independent tables instead of
    per-cell records (ops/fused.py::kernel_geometry): emulated on the host,
    the panel-local record of every window cell, rotated by its panel's
    frame code, reproduces the global record (1/A, centre, curvature sum);
    and in blocks inside one panel the identity-map face lengths and the
    tangent-built line normals equal the plan's per-block tables."""
    from stsphere.ops.fused import global_cell_records, kernel_geometry
    L = TileLayout(N, t, 1, ng=2)
    grid = CubedSphereGrid(N)
    e = Engine(ShallowWater("tc5"), L, grid=grid)
    P = FusedPlan(L, 0, grid, B=B)
    kg = kernel_geometry(L, grid)
    d = P.d
    W, L1, H1 = d.W, d.L1, d.H1
    rec = global_cell_records(e)
    lxt, tane, crec = kg["lxt"], kg["tane"], kg["crec"]
    inner = 0
    for b in range(P.nb):
        X0, Y0 = int(P.org[b, 0]), int(P.org[b, 1])
        for gid in P.gid[b][P.gid[b] >= 0]:
            g, rem = divmod(int(gid), N * N)
            J, I = divmod(rem, N)
            fr = int(kg["frames"][g])
            pi = J * N + I
            assert np.isclose(crec[pi, 0], rec[gid, 0], rtol=1e-13)
            S = _to_global(fr, *crec[pi, 1:4])
            assert np.allclose(S, rec[gid, 7:10], rtol=1e-9, atol=1e-9 * np.abs(rec[gid, 7:10]).max())
            assert np.allclose(_to_global(fr, *crec[pi, 4:7]), rec[gid, 1:4], atol=1e-15)
        if (P.reg[b] != 0).any():
            continue
        inner += 1
        face = L.tile_origin(P.tiles[b // (P.nbx * P.nby)])[0]
        r = np.arange(H1)[:, None]
        c = np.arange(H1 + 1)[None, :]
        assert np.allclose(lxt[Y0 + L1 + r, X0 + L1 + c], P.lx[b], rtol=1e-12)
        assert np.allclose(lxt[X0 + L1 + r, Y0 + L1 + c], P.ly[b].T, rtol=1e-12)
        for ax in (0, 1):
            for k in range(W + 1):
                tn = tane[(Y0 if ax else X0) + k]
                rn = 1.0 / np.sqrt(1 + tn * tn)
                m = _to_global(int(kg["frames"][face]), 0.0 if ax else rn, rn if ax else 0.0, -tn * rn)
                assert np.allclose(m, P.nrm[b, ax, 0, k], atol=1e-14), (b, ax, k)
    assert inner > 0


@pytest.mark.parametrize("N,t,B", [(32, 2, 8), (48, 1, 16), (24, 2, 12)])
def test_fused_loopback_plan_equals_one_rank_cpu(N, t, B):
    """Loopback rehearsal (one rank, layout.loopback): every window cell of
    another tile is a remote cell read from the rank's own ring.  With the
    ring filled from the current state (what the producers' ring stores
    deliver), the PyTorch rendering equals the plain one-rank fused step bit
    for bit, and every ring slot has exactly one producer entry."""
    from stsphere.ops.fused import FusedExchangePlan
    grid = CubedSphereGrid(N)
    L1 = TileLayout(N, t, 1, ng=2)
    one = Engine(ShallowWater("tc5"), L1, grid=grid)
    f1 = FusedTorch(one, FusedPlan(L1, 0, grid, B=B))
    Llb = TileLayout(N, t, 1, ng=2, loopback=True)
    X = FusedExchangePlan(Llb, grid, B)
    assert X.loopback and (X.plans[0].src <= -2).any()
    _, _, pcode = X.producer(0)
    assert sorted(pcode.tolist()) == list(range(len(X.need_remote[0])))
    lb = Engine(ShallowWater("tc5"), Llb, grid=grid, dt=one.dt)
    flb = FusedTorch(lb, X.plans[0], remote_cells=X.need_remote[0])
    off = Llb.local_flat(X.need_remote[0])
    for _ in range(2):
        f1.step()
        recv = lb.pool[0][:, torch.as_tensor(off)].t()
        flb.step(recv)
    assert torch.equal(one.tiles_view(), lb.tiles_view())


@pytest.mark.gpu
@pytest.mark.parametrize("handoff", ["auto", "tag", "epoch"])
@pytest.mark.parametrize("N,t", [(32, 2), (96, 2), (36, 1)])
def test_fused_loopback_kernel_equals_one_rank(monkeypatch, N, t, handoff):
    """The gfx950 fused kernel on a loopback layout (the xGMI ring protocol
    through the rank's own ring, tagged granules every step, one and several
    steps per launch; the in-rank cells by either in-launch hand-off) equals
    the plain one-rank fused step bit for bit."""
    from stsphere.ops.fused import FusedKernel
    monkeypatch.setenv("STSP_FUSED_HANDOFF", handoff)
    grid = CubedSphereGrid(N)
    _, a = _gpu_pair(N, t)
    Llb = TileLayout(N, t, 1, ng=2, loopback=True)
    b = Engine(ShallowWater("tc5"), Llb, grid=grid, dtype=torch.float64, device="cuda", backend="hip", dt=a.dt)
    fa = FusedKernel(a)
    fb = FusedKernel(b, B=fa.plan.B)
    assert fb.mem is not None
    fa.step(3)
    fb.step(3)
    fa.launch(0, nsteps=4)
    fb.launch(0, nsteps=4)
    torch.cuda.synchronize()
    fb.check()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    fb.close()


@pytest.mark.parametrize("N,t,B", [(96, 2, 16), (48, 1, 8), (36, 1, 6), (48, 2, 8), (180, 3, 20)])
def test_block_read_relation_is_symmetric(N, t, B):
    """The tagged in-launch hand-off (two slots, no producer poll) needs every
    reader of a block to be read by it as well, so no producer runs two steps
    ahead of a reader; FusedKernel falls back to the epoch hand-off otherwise."""
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.ops.fused import FusedPlan, read_relation_symmetric
    P = FusedPlan(TileLayout(N, t, 1, ng=2), 0, CubedSphereGrid(N), B=B, ns=3)
    P.src[~P.need[:, 0]] = -1
    assert read_relation_symmetric(P)


@pytest.mark.gpu
@pytest.mark.parametrize("handoff,poll", [("tag", "block"), ("epoch", "cell"), ("epoch", "block")])
@pytest.mark.parametrize("N,t", [(96, 2), (48, 1)])
def test_fused_handoff_forms_equal_single_steps(monkeypatch, handoff, poll, N, t):
    """Every in-launch hand-off form (tagged granules, per-cell producer polls,
    the default block poll), forced on for both block sizes (B = 16 and 8):
    back-to-back multi-step launches, with single steps in between (the epoch
    count pauses), bitwise equal to one launch per step."""
    from stsphere.ops.fused import FusedKernel
    monkeypatch.setenv("STSP_FUSED_HANDOFF", handoff)
    monkeypatch.setenv("STSP_FUSED_POLL", poll)
    _, a = _gpu_pair(N, t)
    _, b = _gpu_pair(N, t)
    b.dt = a.dt
    FusedKernel(a).step(23)
    fk = FusedKernel(b)
    assert fk.handoff == handoff and fk.poll == (poll if handoff == "epoch" else "block")
    fk.launch(0, nsteps=8)
    fk.step(1)
    fk.step(1)
    fk.launch(0, nsteps=6)
    fk.step(1)
    fk.launch(0, nsteps=6)
    torch.cuda.synchronize()
    fk.check()
    assert torch.equal(a.pool[0], b.pool[0])
