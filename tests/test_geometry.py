import math

import numpy as np

from stsphere.models.geometry import CubedSphereGrid, arc_angle


def test_total_area_and_symmetry():
    g = CubedSphereGrid(12)
    assert abs(g.total_area() / (4 * math.pi * g.radius ** 2) - 1) < 1e-13
    a = g.areas()[0]
    assert np.allclose(a, a.T) and np.allclose(a, a[::-1])
    assert 0.70 < a.min() / a.max() < 0.76    # equiangular: -> 1/sqrt(2) as N grows


def test_edge_normals_perpendicular_to_edges_and_unit():
    g = CubedSphereGrid(8)
    v = g.vertices()
    mx = g.x_edge_normals()
    for f in range(6):
        for i in range(9):
            m = mx[f, i]
            assert abs(np.linalg.norm(m) - 1) < 1e-14
            assert np.allclose(v[f, :, i] @ m, 0, atol=1e-14)   # normal to the great circle plane
    my = g.y_edge_normals()
    for f in range(6):
        for j in range(9):
            assert np.allclose(v[f, j, :] @ my[f, j], 0, atol=1e-14)


def test_face3_centre_longitude():
    g = CubedSphereGrid(4)
    lon, lat = g.lonlat()
    assert abs(np.degrees(lon[3]).mean() - 270) < 1e-9    # face 3 centred at 270E (PDF s.13)
    assert np.all(lat[0] > 0.6)                             # face 0 is the north cap


def test_zarr_roundtrip(tmp_path):
    g = CubedSphereGrid(6)
    g.save_zarr(str(tmp_path / "grid.zarr"))
    h = CubedSphereGrid.load_zarr(str(tmp_path / "grid.zarr"))
    assert h.N == 6 and np.array_equal(h.areas(), g.areas())
