"""Host-side index math of the direct xGMI halo (ops/xgmi.py), on CPU.

The data flow of one stage is simulated with numpy: every rank's cells carry
their global id.  Each rank applies its remote push entries into the
receivers' rings.  Then every remote ghost slot of every rank must hold
exactly the cell the geometry says (``ghost_sources``).  The counters' producer
counts and the per-block wait/feed masks are checked against the same
simulation.
"""
import numpy as np
import pytest

from stsphere.ops.xgmi import SLOT_BITS, XgmiPlan, _side_cell
from stsphere.parallel.layout import TileLayout

CASES = [(16, 2, 2, False), (24, 2, 4, False), (16, 2, 8, False), (12, 1, 6, False), (20, 1, 3, False),
         (16, 2, 1, True), (40, 2, 8, False), (36, 3, 6, False)]


def _plans(N, t, R, loop, bx=16, by=16, halo=2):
    L = TileLayout(N, t, R, ng=2, loopback=loop)
    return L, {r: XgmiPlan(L, r, bx, by, halo) for r in range(R)}


@pytest.mark.parametrize("N,t,R,loop", CASES)
def test_every_remote_ghost_delivered(N, t, R, loop):
    L, xp = _plans(N, t, R, loop)
    n = L.n
    ring_slots = xp[0].ring_slots
    assert all(x.ring_slots == ring_slots for x in xp.values())
    rings = {r: np.full(ring_slots, -1, dtype=np.int64) for r in range(R)}
    for r, x in xp.items():
        rem = x.push < -1
        code = (-2 - x.push[rem]).astype(np.int64)
        peer, slot = code >> SLOT_BITS, code & ((1 << SLOT_BITS) - 1)
        li, s2, kk, pp = np.nonzero(rem)
        i, j = _side_cell(s2, kk, pp, n)
        tiles = np.asarray(x.plan.tiles)[li]
        gid = np.empty(len(li), dtype=np.int64)
        for k, tid in enumerate(tiles):
            f, I0, J0 = L.tile_origin(int(tid))
            gid[k] = L.global_flat(f, I0 + i[k], J0 + j[k])
        for p, s, gval in zip(peer, slot, gid):
            assert rings[p][s] in (-1, gval), "two different cells pushed into one ring slot"
            rings[p][s] = gval
        want = set(zip(L.local_flat(gid).tolist(), code.tolist()))
        # carried corner ghosts (panel-edge strip ends): their own push table
        crem = x.cpush < -1
        ccode = (-2 - x.cpush[crem]).astype(np.int64)
        cpeer, cslot = ccode >> SLOT_BITS, ccode & ((1 << SLOT_BITS) - 1)
        cli, cq, ca, cb = np.nonzero(crem)
        ci = np.where(cq & 1, n - 1 - cb, cb)
        cj = np.where(cq & 2, n - 1 - ca, ca)
        for k in range(len(cli)):
            f, I0, J0 = L.tile_origin(int(x.plan.tiles[cli[k]]))
            gval = L.global_flat(f, I0 + ci[k], J0 + cj[k])
            assert rings[cpeer[k]][cslot[k]] in (-1, gval), "two different cells pushed into one ring slot"
            rings[cpeer[k]][cslot[k]] = gval
            want.add((int(L.local_flat(np.array([gval]))[0]), int(ccode[k])))
        # prime entries = the distinct (source cell, destination) pairs of both push tables
        assert len(x.prime_src) == len(np.unique(np.stack([x.prime_src, x.prime_code], 1), axis=0))
        pairs = set(zip(x.prime_src.tolist(), x.prime_code.tolist()))
        assert pairs == want
    ncorner = 0
    for p in range(R):
        pl = L.plan(p)
        gm = pl.ghost_map
        gs = L.ghost_sources(p)
        m = gm < 0
        assert (rings[p][-1 - gm[m]] == gs[m]).all()
        rc = pl.remote_corners()
        ncorner += int(rc.sum())
        assert (rings[p][-1 - pl.corner_map[rc]] == L.corner_sources(p)[rc]).all()
    if t > 1 and R > 1 and not loop:
        assert ncorner > 0 or R <= 2


@pytest.mark.parametrize("N,t,R,loop", CASES)
def test_producer_counts_match_feed_masks(N, t, R, loop):
    L, xp = _plans(N, t, R, loop)
    for r in range(R):
        for p in range(R):
            feeds = int(((xp[p].bmask[:, 1].astype(np.int64) >> r) & 1).sum())
            assert xp[r].nprod[p] == feeds, (r, p)


@pytest.mark.parametrize("N,t,R,loop", CASES)
@pytest.mark.parametrize("halo", [1, 2])
def test_wait_masks_cover_every_window_read(N, t, R, loop, halo):
    """Replays the kernel's window loop (REMOTE branch) for every block."""
    bx = by = 16
    L, xp = _plans(N, t, R, loop, bx, by, halo)
    n = L.n
    for r, x in xp.items():
        plan = x.plan
        gm = plan.ghost_map
        slot_peer = np.full(max(plan.num_recv, 1), -1)
        for p, off, cnt in zip(plan.recv_peers, plan.recv_offsets, plan.recv_counts):
            slot_peer[off:off + cnt] = p
        for bid in range(x.nblocks):
            tile, rem = divmod(bid, x.nbx * x.nby)
            yb, xb = divmod(rem, x.nbx)
            x0, y0 = xb * bx, yb * by
            need = 0
            for ly in range(by + 2 * halo):
                for lx in range(bx + 2 * halo):
                    X, Y = x0 + lx - halo, y0 + ly - halo
                    if not (X < n + halo and Y < n + halo):
                        continue
                    ox, oy = (X < 0) or (X >= n), (Y < 0) or (Y >= n)
                    if ox == oy:
                        continue
                    if X < 0:
                        s, k, pos = 0, -1 - X, Y
                    elif X >= n:
                        s, k, pos = 1, X - n, Y
                    elif Y < 0:
                        s, k, pos = 2, -1 - Y, X
                    else:
                        s, k, pos = 3, Y - n, X
                    m = gm[tile, s, k, pos]
                    if m < 0:
                        need |= 1 << int(slot_peer[-1 - m])
            assert (int(x.bmask[bid, 0]) & need) == need, (r, bid)


def test_single_rank_needs_nothing():
    L, xp = _plans(24, 2, 1, False)
    x = xp[0]
    assert (x.bmask == 0).all() and (x.push >= -1).all() and x.prime_src.size == 0
