"""Cube topology: face frames, edge connectivity, the reference communication
schedule, orientation operators, ghost-cell mapping and edge colouring.

Reference parity
----------------
* ``create_communication_schedule()`` returns exactly the 4-stage x 3-pair table
  of ``JAX-DevLab-Examples.py:105-139`` (PY:114-139).
* ``apply_operations(data, op)`` has the semantics of PY:143-163 on 1-D strips
  ("N"/"T" identity, "R"/"TR" reversal, anything else ``ValueError``), and a
  2-D generalisation (``apply_operations_2d``) for ``ng > 1`` halos where "T"
  is a real (ng x N) -> (N x ng) remap.
* The schedule is *derived* here from geometry (``derive_edge_pairs``) and the
  tests check that the derivation reproduces every op flag of the reference
  table; the reference hard-codes it.
* ``edge_coloring`` is the "general solution: scalable edge coloring" of PDF
  slide 9, used for the staged (debug) communication mode on arbitrary tile /
  device graphs.

Conventions
-----------
Arrays are indexed ``[face, j, i]`` (row j = beta index, column i = alpha
index).  Edge "N" is the last interior row (j = N-1), "S" the first row, "E" the
last column (i = N-1), "W" the first column.  The position along an edge is i
for N/S edges and j for E/W edges, increasing with the index.

Face frames (outward normal n, local east e_i, local north e_j, with
e_i x e_j = n) are the unique right-handed embedding that reproduces every R
flag of the reference schedule.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np

EDGES = ("N", "E", "S", "W")
OPS = ("N", "T", "R", "TR")

# (n, e_i, e_j) per face.  SURVEY.md A.1.
FACE_FRAMES = np.array(
    [
        [[0, 0, 1], [1, 0, 0], [0, 1, 0]],     # 0: top, +z
        [[0, 1, 0], [-1, 0, 0], [0, 0, 1]],    # 1: +y
        [[-1, 0, 0], [0, -1, 0], [0, 0, 1]],   # 2: -x
        [[0, -1, 0], [1, 0, 0], [0, 0, 1]],    # 3: -y
        [[1, 0, 0], [0, 1, 0], [0, 0, 1]],     # 4: +x
        [[0, 0, -1], [-1, 0, 0], [0, 1, 0]],   # 5: bottom, -z
    ],
    dtype=np.float64,
)


def create_communication_schedule():
    """The reference's 12 buffer swaps in 4 stages (PY:105-139), verbatim data.

    Format: ``((face_a, edge_a), (face_b, edge_b), operations)``.
    Each stage is a perfect matching of the 6 faces.
    """
    return (
        (((0, "N"), (1, "N"), "R"), ((3, "E"), (4, "W"), "N"), ((2, "S"), (5, "E"), "TR")),
        (((0, "E"), (4, "N"), "T"), ((2, "E"), (3, "W"), "N"), ((1, "S"), (5, "N"), "N")),
        (((0, "W"), (2, "N"), "TR"), ((1, "W"), (4, "E"), "N"), ((3, "S"), (5, "S"), "R")),
        (((0, "S"), (3, "N"), "N"), ((1, "E"), (2, "W"), "N"), ((4, "S"), (5, "W"), "T")),
    )


def apply_operations(data, operations: str):
    """Orientation operator on a 1-D edge strip (semantics of PY:143-163).

    With a one-cell halo a transposition is realised by extracting a row and
    writing a column, so only the reversal bit acts on the data.
    Works on NumPy arrays and torch tensors.
    """
    if operations in ("N", "T"):
        return data
    if operations in ("R", "TR"):
        return _reverse(data, 0)
    raise ValueError(f"Unknown operation: {operations}")


def apply_operations_2d(strip, operations: str):
    """Orientation operator on a (ng, N) multi-layer strip, layer-major.

    ``strip[k, p]`` is layer k (k = 0 nearest the edge) at edge position p.
    Layers keep their order (depth is preserved across an edge); "R" reverses
    positions.  "T" changes nothing in this layer-major representation: the
    transposition is applied when the strip is *written* (rows <-> columns),
    see ``set_ghost_layers``.
    """
    if operations in ("N", "T"):
        return strip
    if operations in ("R", "TR"):
        return _reverse(strip, strip.ndim - 1)
    raise ValueError(f"Unknown operation: {operations}")


def _reverse(x, dim):
    if hasattr(x, "flip"):  # torch
        return x.flip(dim)
    return np.flip(x, axis=dim)


# ----------------------------------------------------------------------------
# Geometry-derived connectivity
# ----------------------------------------------------------------------------

def _edge_vectors(face: int, edge: str) -> Tuple[np.ndarray, np.ndarray]:
    """(d, a): edge midpoint on the cube is n + d; the edge runs along +a with
    increasing edge position."""
    n, ei, ej = FACE_FRAMES[face]
    if edge == "N":
        return ej, ei
    if edge == "S":
        return -ej, ei
    if edge == "E":
        return ei, ej
    if edge == "W":
        return -ei, ej
    raise ValueError(edge)


@dataclass(frozen=True)
class EdgeLink:
    face: int
    edge: str
    nbr_face: int
    nbr_edge: str
    reversed: bool

    @property
    def transposed(self) -> bool:
        return (self.edge in "NS") != (self.nbr_edge in "NS")

    @property
    def op(self) -> str:
        return ("T" if self.transposed else "") + ("R" if self.reversed else "") or "N"


def _face_of_normal(v: np.ndarray) -> int:
    for f in range(6):
        if np.allclose(FACE_FRAMES[f][0], v):
            return f
    raise AssertionError(v)


def _build_links() -> Dict[Tuple[int, str], EdgeLink]:
    links = {}
    for f in range(6):
        n = FACE_FRAMES[f][0]
        for e in EDGES:
            d, a = _edge_vectors(f, e)
            g = _face_of_normal(d)
            # the neighbour's edge direction vector must be our normal
            ge = None
            for e2 in EDGES:
                d2, a2 = _edge_vectors(g, e2)
                if np.allclose(d2, n):
                    ge = e2
                    rev = bool(np.allclose(a2, -a))
                    assert rev or np.allclose(a2, a)
                    break
            assert ge is not None
            links[(f, e)] = EdgeLink(f, e, g, ge, rev)
    return links


LINKS: Dict[Tuple[int, str], EdgeLink] = _build_links()


def derive_edge_pairs() -> List[Tuple[Tuple[int, str], Tuple[int, str], str]]:
    """The 12 cube edges as ((fa, ea), (fb, eb), op) with fa < fb, derived
    from the face frames (independent of the reference table)."""
    out = []
    for (f, e), lk in sorted(LINKS.items()):
        if f < lk.nbr_face:
            out.append(((f, e), (lk.nbr_face, lk.nbr_edge), lk.op))
    return out


def edge_cell(face_n: int, edge: str, depth: int, pos: int) -> Tuple[int, int]:
    """(i, j) of the interior cell at `depth` (1 = adjacent to the edge) and edge
    position `pos` on an N x N face."""
    N = face_n
    if edge == "N":
        return pos, N - depth
    if edge == "S":
        return pos, depth - 1
    if edge == "E":
        return N - depth, pos
    if edge == "W":
        return depth - 1, pos
    raise ValueError(edge)


def neighbor_cell(N: int, face: int, i: int, j: int) -> Tuple[int, int, int]:
    """Map a cell index of `face` that lies at most one edge outside the face
    (exactly one of i, j out of [0, N)) to the owning (face, i, j).

    Cells beyond a cube corner (both indices outside) have no owner and raise.
    """
    out_i = i < 0 or i >= N
    out_j = j < 0 or j >= N
    if not out_i and not out_j:
        return face, i, j
    if out_i and out_j:
        raise ValueError("cube-corner ghost cell has no owner")
    if j >= N:
        edge, depth, pos = "N", j - N + 1, i
    elif j < 0:
        edge, depth, pos = "S", -j, i
    elif i >= N:
        edge, depth, pos = "E", i - N + 1, j
    else:
        edge, depth, pos = "W", -i, j
    if depth > N:
        raise ValueError("ghost depth exceeds face size")
    lk = LINKS[(face, edge)]
    p2 = N - 1 - pos if lk.reversed else pos
    i2, j2 = edge_cell(N, lk.nbr_edge, depth, p2)
    return lk.nbr_face, i2, j2


def neighbor_cells(N: int, face: int, I: np.ndarray, J: np.ndarray):
    """Vectorised ``neighbor_cell`` for arrays of indices on one face.
    Entries beyond a cube corner get face -1."""
    I = np.asarray(I, dtype=np.int64)
    J = np.asarray(J, dtype=np.int64)
    F = np.full(I.shape, face, dtype=np.int64)
    I2, J2 = I.copy(), J.copy()
    oi = (I < 0) | (I >= N)
    oj = (J < 0) | (J >= N)
    F[oi & oj] = -1
    for edge in EDGES:
        if edge == "N":
            m = (J >= N) & ~oi
            depth, pos = J - N + 1, I
        elif edge == "S":
            m = (J < 0) & ~oi
            depth, pos = -J, I
        elif edge == "E":
            m = (I >= N) & ~oj
            depth, pos = I - N + 1, J
        else:
            m = (I < 0) & ~oj
            depth, pos = -I, J
        if not m.any():
            continue
        lk = LINKS[(face, edge)]
        p2 = np.where(lk.reversed, N - 1 - pos, pos)
        d = depth
        if lk.nbr_edge == "N":
            ii, jj = p2, N - d
        elif lk.nbr_edge == "S":
            ii, jj = p2, d - 1
        elif lk.nbr_edge == "E":
            ii, jj = N - d, p2
        else:
            ii, jj = d - 1, p2
        F[m] = lk.nbr_face
        I2[m] = ii[m]
        J2[m] = jj[m]
    return F, I2, J2


# ----------------------------------------------------------------------------
# Reference-style edge strip helpers (implied API, PY:184-195)
# ----------------------------------------------------------------------------

def boundary_slices(edge: str, N: int, ng: int = 1, layer: int = 0):
    """Index tuple of the interior strip adjacent to `edge` at depth layer+1 in
    a padded (N + 2 ng)^2 face array."""
    lo, hi = ng, ng + N
    if edge == "N":
        return (ng + N - 1 - layer, slice(lo, hi))
    if edge == "S":
        return (ng + layer, slice(lo, hi))
    if edge == "E":
        return (slice(lo, hi), ng + N - 1 - layer)
    if edge == "W":
        return (slice(lo, hi), ng + layer)
    raise ValueError(edge)


def ghost_slices(edge: str, N: int, ng: int = 1, layer: int = 0):
    """Index tuple of the ghost strip beyond `edge` at depth layer+1."""
    lo, hi = ng, ng + N
    if edge == "N":
        return (ng + N + layer, slice(lo, hi))
    if edge == "S":
        return (ng - 1 - layer, slice(lo, hi))
    if edge == "E":
        return (slice(lo, hi), ng + N + layer)
    if edge == "W":
        return (slice(lo, hi), ng - 1 - layer)
    raise ValueError(edge)


# ----------------------------------------------------------------------------
# Edge colouring (PDF s.9: "General solution: scalable edge coloring")
# ----------------------------------------------------------------------------

def edge_coloring(edges: Sequence[Tuple[int, int]], max_colors: int | None = None) -> List[int]:
    """Proper edge colouring of a simple graph: returns one colour per edge so
    that no vertex appears twice in one colour class (one "stage").

    Uses exact backtracking for the minimum (max-degree Delta, falling back to
    Delta + 1, which always exists by Vizing's theorem) on small graphs and the
    greedy bound 2 Delta - 1 as a last resort.  Each colour class is a
    communication stage in which every device talks to at most one partner.
    """
    edges = [tuple(sorted(e)) for e in edges]
    if len(set(edges)) != len(edges):
        raise ValueError("edge_coloring expects a simple graph (bundle parallel edges)")
    if not edges:
        return []
    deg: Dict[int, int] = {}
    for a, b in edges:
        if a == b:
            raise ValueError("self loop")
        deg[a] = deg.get(a, 0) + 1
        deg[b] = deg.get(b, 0) + 1
    delta = max(deg.values())
    order = sorted(range(len(edges)), key=lambda k: -(deg[edges[k][0]] + deg[edges[k][1]]))
    for k in (delta, delta + 1):
        if max_colors is not None and k > max_colors:
            break
        col = _backtrack_coloring(edges, order, k, budget=200000)
        if col is not None:
            return col
    # greedy fallback
    col = [-1] * len(edges)
    used: Dict[int, set] = {v: set() for v in deg}
    for idx in order:
        a, b = edges[idx]
        c = 0
        while c in used[a] or c in used[b]:
            c += 1
        col[idx] = c
        used[a].add(c)
        used[b].add(c)
    return col


def _backtrack_coloring(edges, order, k, budget):
    col = [-1] * len(edges)
    used: Dict[int, set] = {}
    for a, b in edges:
        used.setdefault(a, set())
        used.setdefault(b, set())
    steps = [0]

    def rec(t):
        if t == len(order):
            return True
        steps[0] += 1
        if steps[0] > budget:
            return False
        idx = order[t]
        a, b = edges[idx]
        for c in range(k):
            if c not in used[a] and c not in used[b]:
                col[idx] = c
                used[a].add(c)
                used[b].add(c)
                if rec(t + 1):
                    return True
                used[a].discard(c)
                used[b].discard(c)
                col[idx] = -1
        return False

    return col if rec(0) else None


def coloring_to_stages(edges: Sequence[Tuple[int, int]], colors: Sequence[int]) -> List[List[Tuple[int, int]]]:
    n = max(colors) + 1 if colors else 0
    stages: List[List[Tuple[int, int]]] = [[] for _ in range(n)]
    for e, c in zip(edges, colors):
        stages[c].append(tuple(e))
    return stages


def check_stages(stages) -> bool:
    """True iff no vertex appears twice within any stage (PDF s.9 property)."""
    for st in stages:
        seen = set()
        for a, b in st:
            if a in seen or b in seen:
                return False
            seen.add(a)
            seen.add(b)
    return True


def face_adjacency() -> List[Tuple[int, int]]:
    return [(a[0], b[0]) for a, b, _ in derive_edge_pairs()]


def all_pairs(n: int):
    return list(itertools.combinations(range(n), 2))
