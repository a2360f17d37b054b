"""Tile layout and per-rank halo plans (the "Communication Scheduler" box of
PDF s.7, generalised beyond the reference's fixed 6-face table).

Storage model: every rank holds, per field, its tiles
tile-major with an ng-cell ghost ring, P = n + 2 ng:

    q[field, (tile_local * P + j + ng) * P + i + ng]        interior (i, j) in [0, n)^2

Two maps describe the halo:

    ghost_map[tile_local, side, layer, pos] =  k >= 0   -> q[f, k] (padded offset of the
                                                          same-rank source cell)
                                               -1 - s   -> recv[s, f]  (remote slot s)
    push_map[tile_local, side, layer, pos]  =  padded offset of the ghost slot (in a
                                               same-rank tile) that the interior strip
                                               cell (side, layer, pos) feeds, or -1

The HIP stage kernel *pushes*: when it writes a cell near a tile edge it also
writes the value into the neighbour tile's ghost slot, so the next stage loads
its whole window with plain, regular loads (one memory round trip, no index
indirection).  Remote ghost slots are read from ``recv`` through ghost_map.

with side 0 = W (x < 0), 1 = E (x >= n), 2 = S (y < 0), 3 = N (y >= n), layer
0 nearest the tile edge, pos the index along the edge.  Cross-panel
orientation (the reference's "T"/"R"/"TR" ops, PY:143-163) is folded into the
map, for any halo width ng.

Remote ghost values arrive in ``recv`` (slot-major, fields interleaved:
``recv[slot * F + f]``), one contiguous segment per peer, filled by one RCCL /
gloo message per peer per exchange (bundle per peer).  The
sender packs ``send[k * F + f] = q[f, send_idx[k]]`` in the order the receiver
expects; both sides derive that order from the same deterministic enumeration,
so no index lists are exchanged at run time.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from functools import cached_property
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .partition import partition_tiles, tile_coords, tile_id, tiles_of, validate_device_count
from .topology import neighbor_cells

SIDES = ("W", "E", "S", "N")


def ghost_xy(side: int, layer: int, pos: np.ndarray, n: int):
    """Tile-extended coordinates of ghost cells."""
    if side == 0:
        return np.full_like(pos, -1 - layer), pos
    if side == 1:
        return np.full_like(pos, n + layer), pos
    if side == 2:
        return pos, np.full_like(pos, -1 - layer)
    return pos, np.full_like(pos, n + layer)


def corner_xy(quad, a, b, n: int):
    """Tile-extended coordinates of corner ghost (quad, a, b): quadrant
    quad = (x side E) | 2 (y side N) (0 SW, 1 SE, 2 NW, 3 NE), a rows and b
    columns beyond the tile corner."""
    quad, a, b = np.asarray(quad), np.asarray(a), np.asarray(b)
    x = np.where(quad & 1, n + b, -1 - b)
    y = np.where(quad & 2, n + a, -1 - a)
    return x, y


def corner_own_index(i: np.ndarray, j: np.ndarray, n: int, g: int):
    """Own cell (i, j) inside a g x g tile-corner block -> (quad, a, b), the
    index of the corner push table (the kernels' rule: W / S when the cell is
    within g of both ends, which the layout excludes for carried corners)."""
    qx = np.where(i < g, 0, 1)
    qy = np.where(j < g, 0, 1)
    b = np.where(qx == 0, i, n - 1 - i)
    a = np.where(qy == 0, j, n - 1 - j)
    return qx | (qy << 1), a, b


class TileLayout:
    """Global tiling of a C<N> cubed sphere into 6 t^2 tiles over `num_ranks`."""

    def __init__(self, N: int, tiles_per_edge: int = 1, num_ranks: int = 1, ng: int = 2,
                 partition: str = "auto", owner: Optional[Sequence[int]] = None, loopback: bool = False):
        if N % tiles_per_edge:
            raise ValueError(f"N = {N} is not divisible by tiles_per_edge = {tiles_per_edge}")
        validate_device_count(num_ranks, tiles_per_edge)
        self.N = N
        self.t = tiles_per_edge
        self.n = N // tiles_per_edge
        self.ng = ng
        if ng > self.n:
            raise ValueError(f"halo width ng = {ng} exceeds tile size n = {self.n}")
        self.num_ranks = num_ranks
        # loopback (test/debug): every ghost, even a same-rank one, goes through
        # the pack -> send/recv -> receive-buffer path with the rank as its own peer
        self.loopback = loopback
        self.partition = partition
        self.owner = list(owner) if owner is not None else partition_tiles(tiles_per_edge, num_ranks, partition)
        self.num_tiles = 6 * tiles_per_edge ** 2
        self.rank_tiles: List[List[int]] = [tiles_of(self.owner, r) for r in range(num_ranks)]
        self.local_index: Dict[int, Tuple[int, int]] = {}
        for r, tl in enumerate(self.rank_tiles):
            for li, tid in enumerate(tl):
                self.local_index[tid] = (r, li)
        self._plans: Dict[int, "RankPlan"] = {}
        self._cache: Dict = {}
        self._owner_arr = np.asarray(self.owner, dtype=np.int64)
        self._local_arr = np.zeros(self.num_tiles, dtype=np.int64)
        for tid, (_, li) in self.local_index.items():
            self._local_arr[tid] = li

    # ---- global cell addressing ------------------------------------------
    def tile_origin(self, tid: int) -> Tuple[int, int, int]:
        f, ti, tj = tile_coords(tid, self.t)
        return f, ti * self.n, tj * self.n

    def global_flat(self, face, I, J):
        return (face * self.N + J) * self.N + I

    def tile_extended_index(self, tid: int, ng: Optional[int] = None) -> np.ndarray:
        """[n+2g, n+2g] global flat cell index of every cell in the tile's
        extended (ghosted) window; -1 where undefined (cube-corner ghosts).
        Corner ghosts inside a face (4 tiles meeting) are defined."""
        g = self.ng if ng is None else ng
        n = self.n
        f, I0, J0 = self.tile_origin(tid)
        yy, xx = np.mgrid[-g:n + g, -g:n + g]
        F, I2, J2 = neighbor_cells(self.N, f, I0 + xx, J0 + yy)
        return np.where(F >= 0, self.global_flat(F, I2, J2), -1)

    def locate(self, gflat: np.ndarray):
        """global flat -> (tile_id, i, j)."""
        N, n, t = self.N, self.n, self.t
        face, rem = np.divmod(gflat, N * N)
        J, I = np.divmod(rem, N)
        tid = face * t * t + (J // n) * t + (I // n)
        return tid, I % n, J % n

    # ---- per-rank plans ---------------------------------------------------
    def plan(self, rank: int) -> "RankPlan":
        if rank not in self._plans:
            self._plans[rank] = RankPlan(self, rank)
        return self._plans[rank]

    def ghost_sources(self, rank: int) -> np.ndarray:
        """[T, 4, ng, n] global flat index of the source cell of every ghost."""
        key = ("gs", rank)
        if key in self._cache:
            return self._cache[key]
        tiles = self.rank_tiles[rank]
        n, g = self.n, self.ng
        out = np.empty((len(tiles), 4, g, n), dtype=np.int64)
        pos = np.arange(n)
        for li, tid in enumerate(tiles):
            f, I0, J0 = self.tile_origin(tid)
            for s in range(4):
                for k in range(g):
                    x, y = ghost_xy(s, k, pos, n)
                    F, I2, J2 = neighbor_cells(self.N, f, I0 + x, J0 + y)
                    out[li, s, k] = self.global_flat(F, I2, J2)
        assert (out >= 0).all()
        self._cache[key] = out
        return out

    def corner_sources(self, rank: int) -> np.ndarray:
        """[T, 4, ng, ng] global flat source of the *carried* tile-corner
        ghosts (corner_xy), -1 where none is carried.

        A panel-edge ghost strip is interpolated along the neighbour panel's
        grid lines (models/base.py::panel_edge_tables), whose target points lie
        up to (layer + 1/2) sin(2 beta) cells from the strip cell, toward the
        middle of the panel edge.  Where a tile boundary (not a cube corner)
        cuts the strip, the interpolation pair of the end cells reaches strip
        cells beyond the tile: the diagonal neighbour tile's cells.  Carrying
        them in the tile-corner ghost blocks makes the interpolation, and so
        the state, independent of the decomposition.
        A quadrant whose x side is a panel edge and whose y side is not (or
        the converse) carries its whole ng x ng block: the other panel's
        cells of ghost layers 0 .. ng-1 at the ng strip positions beyond the
        tile end.  Quadrants at a cube corner (both sides on panel edges) and
        inside a panel carry nothing."""
        key = ("cs", rank)
        if key in self._cache:
            return self._cache[key]
        tiles = self.rank_tiles[rank]
        n, g, N = self.n, self.ng, self.N
        out = np.full((len(tiles), 4, g, g), -1, dtype=np.int64)
        for li, tid in enumerate(tiles):
            f, I0, J0 = self.tile_origin(tid)
            for q in range(4):
                xe = (I0 + n == N) if q & 1 else (I0 == 0)
                ye = (J0 + n == N) if q & 2 else (J0 == 0)
                if xe == ye:
                    continue
                if n < 2 * g:
                    raise ValueError(f"tile size n = {n} < 2 ng = {2 * g}: the panel-edge strip ends "
                                     "of a tile boundary cannot be carried")
                a, b = np.meshgrid(np.arange(g), np.arange(g), indexing="ij")
                x, y = corner_xy(q, a, b, n)
                F, I2, J2 = neighbor_cells(N, f, I0 + x, J0 + y)
                assert (F >= 0).all()
                out[li, q, a, b] = self.global_flat(F, I2, J2)
        self._cache[key] = out
        return out

    def needs(self, rank: int, peer: int) -> np.ndarray:
        """Unique global cells owned by `peer` that `rank` reads as ghosts
        (edge strips and carried corner ghosts), in global-id order: the
        producer's row order, so a wave's pushes of one row land in
        consecutive receive slots of the word-major xGMI ring
        (tools/ring_model.py).  Every transport (ring slots, RCCL pack / unpack,
        IPC copies) numbers slots from this one list."""
        cs = self.corner_sources(rank)
        src = np.concatenate([self.ghost_sources(rank).reshape(-1), cs[cs >= 0]])
        tid, _, _ = self.locate(src)
        own = np.asarray(self.owner)[tid]
        return np.unique(src[own == peer])

    def local_flat(self, gflat: np.ndarray) -> np.ndarray:
        """global flat -> padded offset in the owning rank's storage."""
        tid, i, j = self.locate(gflat)
        li = self._local_arr[tid]
        P, g = self.n + 2 * self.ng, self.ng
        return (li * P + j + g) * P + i + g

    def tile_neighbors(self) -> np.ndarray:
        """[num_tiles, 4] tile across side W, E, S, N."""
        key = "tnbr"
        if key not in self._cache:
            n = self.n
            out = np.empty((self.num_tiles, 4), dtype=np.int64)
            for tid in range(self.num_tiles):
                f, I0, J0 = self.tile_origin(tid)
                mid = n // 2
                pts = [(I0 - 1, J0 + mid), (I0 + n, J0 + mid), (I0 + mid, J0 - 1), (I0 + mid, J0 + n)]
                for s, (I, J) in enumerate(pts):
                    F_, I2, J2 = neighbor_cells(self.N, f, np.array([I]), np.array([J]))
                    out[tid, s] = self.locate(self.global_flat(F_, I2, J2))[0][0]
            self._cache[key] = out
        return self._cache[key]


@dataclass
class RankPlan:
    layout: TileLayout
    rank: int

    def __post_init__(self):
        L = self.layout
        self.tiles = list(L.rank_tiles[self.rank])
        self.T = len(self.tiles)
        self.n = L.n
        self.ng = L.ng
        self.P = self.n + 2 * self.ng
        self.S = self.T * self.P * self.P
        src = L.ghost_sources(self.rank)
        csrc = L.corner_sources(self.rank)
        cm = csrc >= 0
        # edge-strip ghosts, then the carried corner ghosts (needs() order)
        allsrc = np.concatenate([src.reshape(-1), csrc[cm]])
        tid, _, _ = L.locate(allsrc)
        own_all = np.asarray(L.owner)[tid]
        codes = np.empty(allsrc.shape, dtype=np.int64)
        local = (own_all == self.rank) & (not L.loopback)
        if local.any():
            codes[local] = L.local_flat(allsrc[local])
        # remote: recv slots, peers in ascending order
        self.recv_peers: List[int] = sorted(int(p) for p in np.unique(own_all[~local]))
        self.recv_counts: List[int] = []
        self.recv_offsets: List[int] = []
        off = 0
        for p in self.recv_peers:
            need = L.needs(self.rank, p)
            m = own_all == p
            sorter = np.argsort(need)
            k = sorter[np.searchsorted(need[sorter], allsrc[m])]
            codes[m] = -1 - (off + k)
            self.recv_offsets.append(off)
            self.recv_counts.append(len(need))
            off += len(need)
        self.num_recv = off
        ns = src.size
        self.ghost_map = codes[:ns].reshape(src.shape).astype(np.int32)
        own = own_all[:ns].reshape(src.shape)
        # corner_map [T, 4, ng, ng], the ghost_map convention for the tile-corner
        # ghost blocks: a carried corner's source (padded offset or -1 - recv
        # slot); any other corner slot names itself (the kernels read it as stored)
        n_, g_, P_ = self.n, self.ng, self.P
        qq, aa, bb = np.meshgrid(np.arange(4), np.arange(g_), np.arange(g_), indexing="ij")
        cx, cy = corner_xy(qq, aa, bb, n_)
        ident = (np.arange(self.T)[:, None, None, None] * P_ + cy[None] + g_) * P_ + cx[None] + g_
        cmap = ident.astype(np.int64)
        cmap[cm] = codes[ns:]
        self.corner_map = cmap.astype(np.int32)
        self.corner_carried = cm
        # send lists: what each peer needs from us, in the peer's order
        self.send_peers: List[int] = []
        self.send_counts: List[int] = []
        self.send_offsets: List[int] = []
        idx = []
        off = 0
        for p in range(L.num_ranks):
            if p == self.rank and not L.loopback:
                continue
            need = L.needs(p, self.rank)
            if len(need) == 0:
                continue
            self.send_peers.append(p)
            self.send_counts.append(len(need))
            self.send_offsets.append(off)
            idx.append(L.local_flat(need))
            off += len(need)
        self.num_send = off
        self.send_idx = (np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)).astype(np.int32)
        self._build_push_map(src, own)

    def _build_push_map(self, src: np.ndarray, own: np.ndarray) -> None:
        """push_map and the halo-refresh index lists (see module docstring)."""
        L = self.layout
        n, g, P, T = self.n, self.ng, self.P, self.T
        tnbr = L.tile_neighbors()
        push = np.full((T, 4, g, n), -1, dtype=np.int64)
        hsrc, hdst = [], []
        pos = np.arange(n)
        for t in range(T):
            for s in range(4):
                for k in range(g):
                    x, y = ghost_xy(s, k, pos, n)
                    dst = (t * P + y + g) * P + x + g
                    loc = (own[t, s, k] == self.rank) & (not L.loopback)
                    if not loc.any():
                        continue
                    c = src[t, s, k][loc]
                    tid2, i2, j2 = L.locate(c)
                    hsrc.append(L.local_flat(c))
                    hdst.append(dst[loc])
                    recv_tile = self.tiles[t]
                    for q, (tt, ii, jj, d) in enumerate(zip(tid2, i2, j2, dst[loc])):
                        sides = np.nonzero(tnbr[tt] == recv_tile)[0]
                        ok = False
                        for s2 in sides:
                            kk, pp = ((ii, jj), (n - 1 - ii, jj), (jj, ii), (n - 1 - jj, ii))[s2]
                            if kk < g:
                                li = L._local_arr[tt]
                                assert push[li, s2, kk, pp] in (-1, d), "push collision"
                                push[li, s2, kk, pp] = d
                                ok = True
                                break
                        assert ok, "no strip feeds this ghost slot"
        self.push_map = push.astype(np.int32)
        # corner_push [T, 4, ng, ng]: the same-rank corner ghost slot (padded
        # offset) that own cell corner_own_index(...) feeds, or -1.  A carried
        # corner's source cell lies in a g x g corner block of its own tile and
        # feeds at most one carried corner (the layout asserts it).
        cpush = np.full((T, 4, g, g), -1, dtype=np.int64)
        cm = self.corner_carried
        cmap = self.corner_map.astype(np.int64)
        if not L.loopback:
            csrc = L.corner_sources(self.rank)
            for t, q, a, b in zip(*np.nonzero(cm & (cmap >= 0))):
                c = csrc[t, q, a, b]
                tid2, i2, j2 = L.locate(np.array([c]))
                assert L.owner[int(tid2[0])] == self.rank
                qo, ao, bo = corner_own_index(i2, j2, n, g)
                x, y = corner_xy(q, a, b, n)
                d = (t * P + int(y) + g) * P + int(x) + g
                key = (int(L._local_arr[tid2[0]]), int(qo[0]), int(ao[0]), int(bo[0]))
                assert cpush[key] in (-1, d), "corner push collision"
                cpush[key] = d
                hsrc.append(np.array([cmap[t, q, a, b]]))
                hdst.append(np.array([d]))
        self.corner_push = cpush.astype(np.int32)
        self.halo_src = (np.concatenate(hsrc) if hsrc else np.zeros(0, np.int64)).astype(np.int32)
        self.halo_dst = (np.concatenate(hdst) if hdst else np.zeros(0, np.int64)).astype(np.int32)

    @property
    def peers(self) -> List[int]:
        return sorted(set(self.recv_peers) | set(self.send_peers))

    def tile_has_remote(self) -> np.ndarray:
        """[T, 4] True where a tile side reads any remote ghost."""
        return (self.ghost_map < 0).any(axis=(2, 3))

    def remote_corners(self) -> np.ndarray:
        """[T, 4, ng, ng] True where a carried corner ghost is a remote one."""
        return self.corner_carried & (self.corner_map < 0)

    def block_classes(self, bx: int, by: int) -> Tuple[np.ndarray, np.ndarray]:
        """Split the (tile, block_y, block_x) work items of a bx x by block
        decomposition into (interior, boundary): boundary blocks read at least
        one remote ghost cell (within `ng` of the block) and must wait for the
        exchange; interior blocks can run while messages are in flight.
        Returns two int32 arrays of linear block ids t*(nby*nbx) + yb*nbx + xb."""
        n, g = self.n, self.ng
        nbx = (n + bx - 1) // bx
        nby = (n + by - 1) // by
        rem = self.ghost_map < 0  # [T,4,g,n]
        interior, boundary = [], []
        rc = self.remote_corners()
        cxy = {}
        for t, q, a, b in zip(*np.nonzero(rc)):
            cxy.setdefault(int(t), []).append(tuple(int(v) for v in corner_xy(q, a, b, n)))
        for t in range(self.T):
            for yb in range(nby):
                y0, y1 = yb * by, min(n, (yb + 1) * by)
                for xb in range(nbx):
                    x0, x1 = xb * bx, min(n, (xb + 1) * bx)
                    r = False
                    if x0 < g and rem[t, 0, : g - x0, y0:y1].any():
                        r = True
                    if x1 > n - g and rem[t, 1, : x1 - (n - g), y0:y1].any():
                        r = True
                    if y0 < g and rem[t, 2, : g - y0, x0:x1].any():
                        r = True
                    if y1 > n - g and rem[t, 3, : y1 - (n - g), x0:x1].any():
                        r = True
                    for (cx, cy) in cxy.get(t, ()):
                        if x0 - g <= cx < x1 + g and y0 - g <= cy < y1 + g:
                            r = True
                    bid = (t * nby + yb) * nbx + xb
                    (boundary if r else interior).append(bid)
        return np.asarray(interior, dtype=np.int32), np.asarray(boundary, dtype=np.int32)

    def summary(self) -> str:
        return (f"rank {self.rank}: tiles {self.tiles}, recv {dict(zip(self.recv_peers, self.recv_counts))}, "
                f"send {dict(zip(self.send_peers, self.send_counts))}")
