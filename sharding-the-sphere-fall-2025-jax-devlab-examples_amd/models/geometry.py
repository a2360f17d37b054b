"""Equiangular gnomonic cubed-sphere geometry (PDF s.4 "Cube Sphere ... Mesh",
s.6 "Geometry: Math/Mesh").

The reference never shows its grid code (appendix A.4 item 11
notes the grid type is unspecified).  This framework fixes it to the
**equiangular gnomonic** grid: on face f with frame (n, e_i, e_j) a point with
local angles (alpha, beta) in [-pi/4, pi/4]^2 is

    r(alpha, beta) = R (n + tan(alpha) e_i + tan(beta) e_j) / |...|.

Everything is computed on the host in float64 and sliced per tile:

* cell centres (unit vectors), latitude / longitude;
* exact cell areas,  A = R^2 [F(X2,Y2) - F(X1,Y2) - F(X2,Y1) + F(X1,Y1)],
  F(X, Y) = atan(X Y / sqrt(1 + X^2 + Y^2)),  X = tan(alpha), Y = tan(beta);
* edge lengths (great-circle arcs between cell vertices);
* edge unit normals.  Lines of constant alpha are great circles, so the in-
  surface normal of an x-edge is the same along the whole edge and depends on
  the column only:  m_x = (e_i - X n) / sqrt(1 + X^2)  (points to +alpha);
  likewise m_y = (e_j - Y n) / sqrt(1 + Y^2).

Arrays are ``[face, j, i, ...]``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

from ..parallel.topology import FACE_FRAMES

EARTH_RADIUS = 6.37122e6
OMEGA = 7.292e-5
GRAVITY = 9.80616
DAY = 86400.0


def _area_F(X, Y):
    return np.arctan(X * Y / np.sqrt(1.0 + X * X + Y * Y))


def face_points(X: np.ndarray, Y: np.ndarray) -> np.ndarray:
    """Unit vectors for all faces: X, Y broadcastable arrays of tan(angle).
    Returns [6, *broadcast_shape, 3]."""
    X, Y = np.broadcast_arrays(np.asarray(X, dtype=np.float64), np.asarray(Y, dtype=np.float64))
    ei =FACE_FRAMES[:, 1].reshape((6,) + (1,) * X.ndim + (3,))
    ej = FACE_FRAMES[:, 2].reshape((6,) + (1,) * X.ndim + (3,))
    n = FACE_FRAMES[:, 0].reshape((6,) + (1,) * X.ndim + (3,))
    p = n + X[None, ..., None] * ei + Y[None, ..., None] * ej
    return p / np.linalg.norm(p, axis=-1, keepdims=True)


def arc_angle(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Great-circle angle between unit vectors (last axis)."""
    c = np.cross(a, b)
    return np.arctan2(np.linalg.norm(c, axis=-1), np.sum(a * b, axis=-1))


def xyz_to_lonlat(p: np.ndarray):
    lon = np.mod(np.arctan2(p[..., 1], p[..., 0]), 2 * np.pi)
    lat = np.arcsin(np.clip(p[..., 2], -1.0, 1.0))
    return lon, lat


def lonlat_to_xyz(lon, lat):
    return np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], axis=-1)


@dataclass
class CubedSphereGrid:
    """Global C<N> equiangular grid, float64, radius R."""

    N: int
    radius: float = EARTH_RADIUS
    _cache: Dict[str, np.ndarray] = field(default_factory=dict, repr=False)

    @property
    def dalpha(self) -> float:
        return 0.5 * math.pi / self.N

    def alpha_edges(self) -> np.ndarray:
        return -0.25 * math.pi + self.dalpha * np.arange(self.N + 1)

    def alpha_centers(self) -> np.ndarray:
        return -0.25 * math.pi + self.dalpha * (np.arange(self.N) + 0.5)

    def _get(self, key, fn):
        if key not in self._cache:
            self._cache[key] = fn()
        return self._cache[key]

    # ---- points --------------------------------------------------------
    def vertices(self) -> np.ndarray:
        """[6, N+1, N+1, 3] unit vectors of cell corners ([face, j, i])."""
        def f():
            Xe = np.tan(self.alpha_edges())
            return face_points(Xe[None, :], Xe[:, None])
        return self._get("vertices", f)

    def centers(self) -> np.ndarray:
        """[6, N, N, 3] unit vectors of cell centres (equiangular midpoint)."""
        def f():
            Xc = np.tan(self.alpha_centers())
            return face_points(Xc[None, :], Xc[:, None])
        return self._get("centers", f)

    def lonlat(self):
        c = self.centers()
        return xyz_to_lonlat(c)

    # ---- metrics -------------------------------------------------------
    def areas(self) -> np.ndarray:
        """[6, N, N] exact spherical cell areas (m^2)."""
        def f():
            Xe = np.tan(self.alpha_edges())
            F = _area_F(Xe[None, :], Xe[:, None])  # [j, i]
            a = F[1:, 1:] - F[1:, :-1] - F[:-1, 1:] + F[:-1, :-1]
            return np.broadcast_to(a * self.radius ** 2, (6, self.N, self.N)).copy()
        return self._get("areas", f)

    def x_edge_lengths(self) -> np.ndarray:
        """[6, N, N+1]: length of the edge at column i' between rows j, j+1."""
        def f():
            v = self.vertices()
            return arc_angle(v[:, :-1, :, :], v[:, 1:, :, :]) * self.radius
        return self._get("lx", f)

    def y_edge_lengths(self) -> np.ndarray:
        """[6, N+1, N]: length of the edge at row j' between columns i, i+1."""
        def f():
            v = self.vertices()
            return arc_angle(v[:, :, :-1, :], v[:, :, 1:, :]) * self.radius
        return self._get("ly", f)

    def x_edge_normals(self) -> np.ndarray:
        """[6, N+1, 3] unit normal of x-edges (column i'), pointing to +alpha."""
        def f():
            X = np.tan(self.alpha_edges())
            n = FACE_FRAMES[:, 0][:, None, :]
            ei = FACE_FRAMES[:, 1][:, None, :]
            m = ei - X[None, :, None] * n
            return m / np.sqrt(1 + X * X)[None, :, None]
        return self._get("mx", f)

    def y_edge_normals(self) -> np.ndarray:
        """[6, N+1, 3] unit normal of y-edges (row j'), pointing to +beta."""
        def f():
            Y = np.tan(self.alpha_edges())
            n = FACE_FRAMES[:, 0][:, None, :]
            ej = FACE_FRAMES[:, 2][:, None, :]
            m = ej - Y[None, :, None] * n
            return m / np.sqrt(1 + Y * Y)[None, :, None]
        return self._get("my", f)

    def x_edge_midpoints(self) -> np.ndarray:
        """[6, N, N+1, 3] unit vectors of x-edge midpoints."""
        def f():
            v = self.vertices()
            m = v[:, :-1, :, :] + v[:, 1:, :, :]
            return m / np.linalg.norm(m, axis=-1, keepdims=True)
        return self._get("xmid", f)

    def y_edge_midpoints(self) -> np.ndarray:
        def f():
            v = self.vertices()
            m = v[:, :, :-1, :] + v[:, :, 1:, :]
            return m / np.linalg.norm(m, axis=-1, keepdims=True)
        return self._get("ymid", f)

    def total_area(self) -> float:
        return float(self.areas().sum())

    def min_spacing(self) -> float:
        return float(min(self.x_edge_lengths().min(), self.y_edge_lengths().min()))

    def to_arrays(self) -> Dict[str, np.ndarray]:
        """All geometry arrays, for zarr export (PDF s.6 'Geometry: jax.zarr')."""
        lon, lat = self.lonlat()
        return {
            "centers": self.centers(),
            "vertices": self.vertices(),
            "areas": self.areas(),
            "lon": lon,
            "lat": lat,
            "x_edge_lengths": self.x_edge_lengths(),
            "y_edge_lengths": self.y_edge_lengths(),
            "x_edge_normals": self.x_edge_normals(),
            "y_edge_normals": self.y_edge_normals(),
            "x_edge_midpoints": self.x_edge_midpoints(),
            "y_edge_midpoints": self.y_edge_midpoints(),
        }

    _ZARR_KEYS = {"centers": "centers", "vertices": "vertices", "areas": "areas", "x_edge_lengths": "lx",
                  "y_edge_lengths": "ly", "x_edge_normals": "mx", "y_edge_normals": "my",
                  "x_edge_midpoints": "xmid", "y_edge_midpoints": "ymid"}

    def save_zarr(self, path: str) -> None:
        from ..utils import zarr_lite
        g = zarr_lite.create_group(path, attrs={"grid": "equiangular_gnomonic", "N": self.N, "radius": self.radius})
        for k, v in self.to_arrays().items():
            zarr_lite.write_array(path, k, v)

    @classmethod
    def load_zarr(cls, path: str, N: Optional[int] = None, radius: Optional[float] = None) -> "CubedSphereGrid":
        """Grid whose arrays are read from a zarr group written by
        ``save_zarr`` (the pipeline's Geometry stage, PDF s.6).  ``N`` /
        ``radius``, when given, must match the stored grid."""
        from ..utils import zarr_lite
        attrs = zarr_lite.read_attrs(path)
        if attrs.get("grid") != "equiangular_gnomonic":
            raise ValueError(f"{path}: not an equiangular gnomonic grid ({attrs.get('grid')!r})")
        g = cls(int(attrs["N"]), float(attrs["radius"]))
        if N is not None and g.N != N:
            raise ValueError(f"{path}: stored grid is C{g.N}, config asks for C{N}")
        if radius is not None and g.radius != radius:
            raise ValueError(f"{path}: stored radius {g.radius} != configured {radius}")
        have = set(zarr_lite.list_arrays(path))
        for k, key in cls._ZARR_KEYS.items():
            if k in have:
                g._cache[key] = zarr_lite.read_array(path, k)
        return g


def tangent_project(v: np.ndarray, r: np.ndarray) -> np.ndarray:
    return v - np.sum(v * r, axis=-1, keepdims=True) * r


def lonlat_vectors(p: np.ndarray):
    """Unit east / north vectors at unit positions p [...,3]."""
    lon, lat = xyz_to_lonlat(p)
    east = np.stack([-np.sin(lon), np.cos(lon), np.zeros_like(lon)], axis=-1)
    north = np.stack([-np.sin(lat) * np.cos(lon), -np.sin(lat) * np.sin(lon), np.cos(lat)], axis=-1)
    return east, north


def wind_cartesian(p: np.ndarray, u: np.ndarray, v: np.ndarray) -> np.ndarray:
    """Cartesian wind from zonal u / meridional v at positions p."""
    e, n = lonlat_vectors(p)
    return u[..., None] * e + v[..., None] * n
