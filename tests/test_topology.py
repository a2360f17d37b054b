"""Cube topology vs the reference schedule (PY:105-139) and PDF s.9 properties."""
import numpy as np
import pytest

from stsphere.parallel import topology as T


def test_schedule_is_reference_table():
    s = T.create_communication_schedule()
    assert len(s) == 4 and all(len(st) == 3 for st in s)
    assert s[0][0] == ((0, "N"), (1, "N"), "R")
    assert s[3][2] == ((4, "S"), (5, "W"), "T")


def test_derived_geometry_reproduces_every_op():
    derived = {(a, b): op for a, b, op in T.derive_edge_pairs()}
    assert len(derived) == 12
    for st in T.create_communication_schedule():
        for a, b, op in st:
            key = (a, b) if (a, b) in derived else (b, a)
            assert derived[key] == op


def test_each_stage_is_perfect_matching_and_edges_used_once():
    used = set()
    for st in T.create_communication_schedule():
        faces = [a[0] for a, b, _ in st] + [b[0] for a, b, _ in st]
        assert sorted(faces) == list(range(6))          # no device twice per stage (PDF s.9)
        for a, b, _ in st:
            used.add(a)
            used.add(b)
    assert used == {(f, e) for f in range(6) for e in "NESW"}


def test_frames_right_handed_and_opposites():
    for f in range(6):
        n, ei, ej = T.FACE_FRAMES[f]
        assert np.allclose(np.cross(ei, ej), n)
    for a, b in ((0, 5), (1, 3), (2, 4)):
        assert np.allclose(T.FACE_FRAMES[a][0], -T.FACE_FRAMES[b][0])


def test_transpose_iff_row_meets_column():
    for (f, e), lk in T.LINKS.items():
        assert lk.transposed == ((e in "NS") != (lk.nbr_edge in "NS"))
        back = T.LINKS[(lk.nbr_face, lk.nbr_edge)]
        assert (back.nbr_face, back.nbr_edge) == (f, e) and back.reversed == lk.reversed


def test_apply_operations_semantics():
    d = np.arange(5)
    assert (T.apply_operations(d, "N") == d).all()
    assert (T.apply_operations(d, "T") == d).all()
    assert (T.apply_operations(d, "R") == d[::-1]).all()
    assert (T.apply_operations(d, "TR") == d[::-1]).all()
    with pytest.raises(ValueError, match="Unknown operation"):
        T.apply_operations(d, "X")


def test_neighbor_cell_roundtrip():
    N = 7
    for f in range(6):
        for edge in "NESW":
            for depth in (1, 2, 3):
                for p in range(N):
                    i, j = {"N": (p, N - 1 + depth), "S": (p, -depth), "E": (N - 1 + depth, p), "W": (-depth, p)}[edge]
                    g, i2, j2 = T.neighbor_cell(N, f, i, j)
                    assert 0 <= i2 < N and 0 <= j2 < N and g != f
                    G, I2, J2 = T.neighbor_cells(N, f, np.array([i]), np.array([j]))
                    assert (G[0], I2[0], J2[0]) == (g, i2, j2)


def test_edge_coloring_octahedron_and_cube_graph():
    octa = T.face_adjacency()
    c = T.edge_coloring(octa)
    stages = T.coloring_to_stages(octa, c)
    assert len(stages) == 4 and T.check_stages(stages)
    cube = [(a, b) for a in range(8) for b in range(a + 1, 8) if bin(a ^ b).count("1") == 1]
    st = T.coloring_to_stages(cube, T.edge_coloring(cube))
    assert len(st) == 3 and T.check_stages(st)
    k5 = T.all_pairs(5)
    st = T.coloring_to_stages(k5, T.edge_coloring(k5))
    assert len(st) == 5 and T.check_stages(st)   # class-2 graph: Delta + 1
