"""Halo maps checked geometrically, independently of the map construction
(every ghost must hold the geometrically adjacent cell)."""
import numpy as np
import pytest

from stsphere.models.geometry import CubedSphereGrid
from stsphere.parallel.layout import TileLayout, ghost_xy


def _cell_vertex_sets(N):
    g = CubedSphereGrid(N, radius=1.0)
    v = g.vertices()
    key = {}
    ids = np.empty(v.shape[:3], dtype=np.int64)
    for idx in np.ndindex(*v.shape[:3]):
        k = tuple(np.round(v[idx], 9))
        ids[idx] = key.setdefault(k, len(key))
    assert len(key) == 6 * N * N + 2          # Euler: V = 6N^2 + 2
    cells = {}
    for f in range(6):
        for j in range(N):
            for i in range(N):
                cells[(f * N + j) * N + i] = frozenset((ids[f, j, i], ids[f, j, i + 1], ids[f, j + 1, i], ids[f, j + 1, i + 1]))
    return cells


def _adjacent(cells, a, b):
    return len(cells[a] & cells[b]) == 2


@pytest.mark.parametrize("N,t,ng", [(6, 1, 2), (8, 2, 3), (9, 3, 2), (4, 1, 3)])
def test_ghost_sources_are_geometric_neighbours(N, t, ng):
    L = TileLayout(N, t, 1, ng=ng)
    cells = _cell_vertex_sets(N)
    src = L.ghost_sources(0)   # [T,4,ng,n]
    n = L.n
    for li, tid in enumerate(L.rank_tiles[0]):
        f, I0, J0 = L.tile_origin(tid)
        for s in range(4):
            for p in range(n):
                # tile boundary cell adjacent to this side at position p
                x, y = ghost_xy(s, 0, np.array([p]), n)
                bx = min(max(int(x[0]), 0), n - 1)
                by = min(max(int(y[0]), 0), n - 1)
                inner = L.global_flat(f, I0 + bx, J0 + by)
                prev, prev2 = inner, None
                for k in range(ng):
                    c = int(src[li, s, k, p])
                    assert _adjacent(cells, c, prev), (tid, s, k, p)
                    assert c != prev2
                    if k >= 1:
                        assert not _adjacent(cells, c, inner)
                    if p + 1 < n:
                        assert _adjacent(cells, c, int(src[li, s, k, p + 1]))
                    prev2, prev = prev, c


@pytest.mark.parametrize("N,t,R", [(8, 2, 8), (12, 2, 4), (12, 1, 3), (8, 2, 2)])
def test_send_recv_lists_consistent(N, t, R):
    L = TileLayout(N, t, R, ng=2)
    for r in range(R):
        p = L.plan(r)
        for peer, off, cnt in zip(p.recv_peers, p.recv_offsets, p.recv_counts):
            q = L.plan(peer)
            k = q.send_peers.index(r)
            assert q.send_counts[k] == cnt
            # sender's cells (padded offsets -> global) are exactly what r needs, in order
            need = L.needs(r, peer)
            sent = q.send_idx[q.send_offsets[k]:q.send_offsets[k] + cnt]
            assert (L.local_flat(need) == sent).all()
        # every remote ghost references a valid slot
        gm = p.ghost_map
        assert ((-1 - gm[gm < 0]) < p.num_recv).all()


@pytest.mark.parametrize("N,t,R", [(8, 1, 1), (8, 2, 1), (12, 2, 8)])
def test_push_map_is_bijection_onto_local_ghosts(N, t, R):
    L = TileLayout(N, t, R, ng=2)
    for r in range(R):
        p = L.plan(r)
        pushed = p.push_map[p.push_map >= 0]
        assert len(np.unique(pushed)) == len(pushed) == (p.ghost_map >= 0).sum()
        # carried corner ghosts: pushed by their own table, once each
        cp = p.corner_push[p.corner_push >= 0]
        assert len(np.unique(cp)) == len(cp) == (p.corner_carried & (p.corner_map >= 0)).sum()
        allp = np.concatenate([pushed, cp])
        assert len(np.unique(allp)) == len(allp)
        assert set(allp.tolist()) == set(p.halo_dst.tolist())


@pytest.mark.parametrize("N,t,R,ng", [(12, 2, 1, 2), (24, 4, 1, 3), (24, 2, 6, 2), (24, 4, 8, 3)])
def test_corner_ghosts_carry_the_diagonal_strip_cells(N, t, R, ng):
    """Carried corner ghosts: exactly the quadrants with one panel-edge side,
    each slot's source is the true neighbour-panel cell at that extended
    position (tile_extended_index), and every remote one has a receive slot
    whose sender packs that cell."""
    L = TileLayout(N, t, R, ng=ng)
    n = L.n
    for r in range(R):
        p = L.plan(r)
        cs = L.corner_sources(r)
        for li, tid in enumerate(p.tiles):
            f, I0, J0 = L.tile_origin(tid)
            ext = L.tile_extended_index(tid, ng)
            for q in range(4):
                xe = (I0 + n == N) if q & 1 else (I0 == 0)
                ye = (J0 + n == N) if q & 2 else (J0 == 0)
                assert p.corner_carried[li, q].all() == (xe != ye)
                assert p.corner_carried[li, q].any() == (xe != ye)
                for a in range(ng):
                    for b in range(ng):
                        x = n + b if q & 1 else -1 - b
                        y = n + a if q & 2 else -1 - a
                        if xe != ye:
                            assert cs[li, q, a, b] == ext[y + ng, x + ng] >= 0
        rc = p.remote_corners()
        if rc.any():
            slots = -1 - p.corner_map[rc]
            assert (slots < p.num_recv).all()
            for s, c in zip(slots, cs[rc]):
                k = int(np.searchsorted(np.asarray(p.recv_offsets), s, side="right")) - 1
                peer = p.recv_peers[k]
                assert L.needs(r, peer)[s - p.recv_offsets[k]] == c


def test_block_classes_partition_all_blocks():
    L = TileLayout(64, 2, 8, ng=2)
    p = L.plan(0)
    inter, bnd = p.block_classes(16, 16)
    allb = np.sort(np.concatenate([inter, bnd]))
    assert (allb == np.arange(p.T * 2 * 2)).all() and len(bnd) > 0 and len(inter) > 0
