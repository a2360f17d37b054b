"""Graph partitioner: cubed-sphere tiles -> devices (PDF s.7 "Graph Partitioner").

The reference only has the implicit contiguous block split of axis 0 done by
``NamedSharding(mesh, P('tiles'))`` (PY:77-79) and rejects ``tiles_per_edge != 1``
(PY:31-37).  Here ``tiles_per_edge = t >= 1`` is supported (6 t^2 tiles of
(N/t)^2 cells) and three strategies exist:

* ``contiguous`` -- the reference semantics: device d owns tiles
  [d*k, (d+1)*k), k = 6 t^2 / num_devices.
* ``corner``     -- for even t and 2/4/8 devices: the 3 face-quadrants around each
  cube vertex form a group; 8 groups -> 8 devices (cube graph, 3 peers per
  device, 24 of 48 tile edges cut at t=2), pairs of groups along a vertical cube
  edge -> 4 devices, top/bottom halves -> 2 devices.
* ``auto``       -- corner where it applies, else contiguous.

Validation mirrors PY:40-57 (same errors and message text for bad counts).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from .topology import FACE_FRAMES, neighbor_cell


def num_tiles(tiles_per_edge: int) -> int:
    return 6 * tiles_per_edge * tiles_per_edge


def valid_device_counts(tiles_per_edge: int) -> List[int]:
    nt = num_tiles(tiles_per_edge)
    return [d for d in range(1, nt + 1) if nt % d == 0]


def validate_device_count(num_devices: int, tiles_per_edge: int) -> int:
    """Raise exactly like PY:43-57; return num_tiles."""
    if tiles_per_edge < 1:
        raise ValueError(f"Error: tiles_per_edge = {tiles_per_edge} must be >= 1.")
    nt = num_tiles(tiles_per_edge)
    if num_devices > nt:
        raise ValueError(
            f"Error: num_devices = {num_devices} exceeds num_tiles = {nt}.\n"
            f"Cannot have more devices than tiles.\n"
            f"With tiles_per_edge = {tiles_per_edge}, max devices = {nt}."
        )
    if nt % num_devices != 0:
        valid_counts = valid_device_counts(tiles_per_edge)
        raise ValueError(
            f"Error: num_tiles = {nt} is not evenly divisible by num_devices = {num_devices}.\n"
            f"Tile sharding requires: num_tiles % num_devices == 0\n"
            f"With tiles_per_edge = {tiles_per_edge}, valid device counts are:\n"
            f"  {valid_counts}"
        )
    return nt


def tile_id(face: int, ti: int, tj: int, t: int) -> int:
    return face * t * t + tj * t + ti


def tile_coords(tid: int, t: int) -> Tuple[int, int, int]:
    face, r = divmod(tid, t * t)
    tj, ti = divmod(r, t)
    return face, ti, tj


def tile_adjacency(t: int) -> List[Tuple[int, int]]:
    """The 12 t^2 tile edges as (tile_a, tile_b) pairs with a < b (each tile
    edge once).  Uses the cell-level neighbour map on a face of N = t cells, so
    each cell is a tile."""
    pairs = set()
    for f in range(6):
        for tj in range(t):
            for ti in range(t):
                a = tile_id(f, ti, tj, t)
                for di, dj in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                    g, i2, j2 = neighbor_cell(t, f, ti + di, tj + dj)
                    b = tile_id(g, i2, j2, t)
                    pairs.add((min(a, b), max(a, b)))
    return sorted(pairs)


def _corner_key(face: int, ti: int, tj: int, t: int) -> Tuple[int, int, int]:
    n, ei, ej = FACE_FRAMES[face]
    sa = 1 if ti >= t // 2 else -1
    sb = 1 if tj >= t // 2 else -1
    v = n + sa * ei + sb * ej
    return tuple(int(round(x)) for x in v)


CORNERS = [(sx, sy, sz) for sz in (1, -1) for sy in (1, -1) for sx in (1, -1)]


def partition_tiles(tiles_per_edge: int, num_devices: int, strategy: str = "auto") -> List[int]:
    """owner[tile_id] = device index."""
    t = tiles_per_edge
    nt = validate_device_count(num_devices, t)
    if strategy == "auto":
        strategy = "corner" if (t % 2 == 0 and num_devices in (2, 4, 8)) else "contiguous"
    if strategy == "contiguous":
        k = nt // num_devices
        return [tid // k for tid in range(nt)]
    if strategy == "corner":
        if t % 2 != 0 or num_devices not in (1, 2, 4, 8):
            raise ValueError("corner partition needs even tiles_per_edge and 1/2/4/8 devices")
        owner = []
        for tid in range(nt):
            f, ti, tj = tile_coords(tid, t)
            c = _corner_key(f, ti, tj, t)
            sx, sy, sz = c
            if num_devices == 8:
                d = CORNERS.index(c)
            elif num_devices == 4:
                d = [(1, 1), (-1, 1), (-1, -1), (1, -1)].index((sx, sy))  # vertical cube edges, ring order
            elif num_devices == 2:
                d = 0 if sz > 0 else 1
            else:
                d = 0
            owner.append(d)
        return owner
    raise ValueError(f"unknown partition strategy {strategy!r}")


def cut_edges(tiles_per_edge: int, owner: Sequence[int]) -> int:
    return sum(1 for a, b in tile_adjacency(tiles_per_edge) if owner[a] != owner[b])


def device_graph(tiles_per_edge: int, owner: Sequence[int]) -> Dict[Tuple[int, int], int]:
    """{(dev_a, dev_b): number of tile edges between them} for a < b."""
    g: Dict[Tuple[int, int], int] = {}
    for a, b in tile_adjacency(tiles_per_edge):
        da, db = owner[a], owner[b]
        if da != db:
            k = (min(da, db), max(da, db))
            g[k] = g.get(k, 0) + 1
    return g


def partition_report(tiles_per_edge: int, owner: Sequence[int]) -> str:
    nd = max(owner) + 1
    g = device_graph(tiles_per_edge, owner)
    peers = {d: sorted({b if a == d else a for (a, b) in g if d in (a, b)}) for d in range(nd)}
    lines = [f"    cut tile edges: {cut_edges(tiles_per_edge, owner)} / {len(tile_adjacency(tiles_per_edge))}"]
    for d in range(nd):
        tiles = [i for i, o in enumerate(owner) if o == d]
        lines.append(f"    device {d}: tiles {tiles} peers {peers[d]}")
    return "\n".join(lines)


def tiles_of(owner: Sequence[int], device: int) -> List[int]:
    return [i for i, o in enumerate(owner) if o == device]


def balance(owner: Sequence[int]) -> np.ndarray:
    return np.bincount(np.asarray(owner))
