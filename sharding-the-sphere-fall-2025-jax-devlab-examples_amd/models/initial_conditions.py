"""Initial conditions / physics setups (PDF s.6 "Initial Conditions: Physics").

All functions take unit position vectors ``p[..., 3]`` and return NumPy float64
arrays; winds are returned as **Cartesian** (x, y, z) vectors, the panel-
invariant representation the reference exchanges across cube edges (PDF s.18
"Cartesian Velocity Exchange").

* ``cosine_bell``       Williamson et al. (1992) test case 1 (PDF s.13 / s.18:
                        bell at 270 E, 0 N, peak ~1000).
* ``solid_body_wind``   TC1/TC2 wind, rotation angle alpha.
* ``williamson_tc2``    steady geostrophic flow (analytic solution = IC).
* ``williamson_tc5``    zonal flow over an isolated mountain.
* ``williamson_tc6``    Rossby-Haurwitz wave, wavenumber 4.
* ``lima_flag``         checkerboard heat source on the top panel (face 0) on a
                        1 K background (PDF s.12 / s.17, log scale 1..1000 K).
"""
from __future__ import annotations

import math

import numpy as np

from .geometry import DAY, EARTH_RADIUS, GRAVITY, OMEGA, lonlat_vectors, xyz_to_lonlat


def great_circle_distance(lon1, lat1, lon2, lat2, radius=EARTH_RADIUS):
    c = np.sin(lat1) * np.sin(lat2) + np.cos(lat1) * np.cos(lat2) * np.cos(lon1 - lon2)
    return radius * np.arccos(np.clip(c, -1.0, 1.0))


def solid_body_wind(p, u0=None, alpha=0.0, radius=EARTH_RADIUS):
    """Williamson TC1/TC2 wind: u = u0 (cos phi cos a + sin phi cos lam sin a),
    v = -u0 sin lam sin a.  Returned as Cartesian vectors."""
    if u0 is None:
        u0 = 2.0 * math.pi * radius / (12.0 * DAY)
    lon, lat = xyz_to_lonlat(p)
    u = u0 * (np.cos(lat) * math.cos(alpha) + np.sin(lat) * np.cos(lon) * math.sin(alpha))
    v = -u0 * np.sin(lon) * math.sin(alpha)
    e, n = lonlat_vectors(p)
    return u[..., None] * e + v[..., None] * n


def rotated_center(lon_c, lat_c, t, alpha, u0, radius=EARTH_RADIUS):
    """Position of the TC1 bell centre after time t (solid-body rotation
    about the axis tilted by alpha)."""
    w = u0 / radius
    # rotation axis: Omega_vec such that v = w x r reproduces solid_body_wind
    axis = np.array([-math.sin(alpha), 0.0, math.cos(alpha)])
    c0 = np.array([math.cos(lat_c) * math.cos(lon_c), math.cos(lat_c) * math.sin(lon_c), math.sin(lat_c)])
    th = w * t
    # Rodrigues
    c = (c0 * math.cos(th) + np.cross(axis, c0) * math.sin(th) + axis * np.dot(axis, c0) * (1 - math.cos(th)))
    return c


def cosine_bell(p, h0=1000.0, lon_c=1.5 * math.pi, lat_c=0.0, r0=None, radius=EARTH_RADIUS, center_xyz=None):
    if r0 is None:
        r0 = radius / 3.0
    lon, lat = xyz_to_lonlat(p)
    if center_xyz is not None:
        cc = np.asarray(center_xyz)
        lat_c = math.asin(max(-1.0, min(1.0, cc[2])))
        lon_c = math.atan2(cc[1], cc[0]) % (2 * math.pi)
    r = great_circle_distance(lon, lat, lon_c, lat_c, radius)
    return np.where(r < r0, 0.5 * h0 * (1.0 + np.cos(math.pi * r / r0)), 0.0)


def cosine_bell_exact(p, t, alpha=0.0, h0=1000.0, radius=EARTH_RADIUS, u0=None):
    if u0 is None:
        u0 = 2.0 * math.pi * radius / (12.0 * DAY)
    c = rotated_center(1.5 * math.pi, 0.0, t, alpha, u0, radius)
    return cosine_bell(p, h0=h0, radius=radius, center_xyz=c)


def williamson_tc2(p, alpha=0.0, gh0=2.94e4, radius=EARTH_RADIUS, omega=OMEGA, g=GRAVITY):
    """Returns (h, wind, b).  Steady state: h(t) = h(0)."""
    u0 = 2.0 * math.pi * radius / (12.0 * DAY)
    lon, lat = xyz_to_lonlat(p)
    s = -np.cos(lon) * np.cos(lat) * math.sin(alpha) + np.sin(lat) * math.cos(alpha)
    gh = gh0 - (radius * omega * u0 + 0.5 * u0 * u0) * s * s
    wind = solid_body_wind(p, u0, alpha, radius)
    return gh / g, wind, np.zeros_like(gh)


def tc5_mountain(p, hs0=2000.0, lon_c=1.5 * math.pi, lat_c=math.pi / 6.0, Rm=math.pi / 9.0):
    lon, lat = xyz_to_lonlat(p)
    dl = np.mod(lon - lon_c + math.pi, 2 * math.pi) - math.pi
    r = np.minimum(Rm, np.sqrt(dl * dl + (lat - lat_c) ** 2))
    return hs0 * (1.0 - r / Rm)


def williamson_tc5(p, h0=5960.0, u0=20.0, radius=EARTH_RADIUS, omega=OMEGA, g=GRAVITY):
    """Zonal flow over an isolated mountain.  Returns (h = fluid depth, wind, b)."""
    lon, lat = xyz_to_lonlat(p)
    b = tc5_mountain(p)
    htot = h0 - (radius * omega * u0 + 0.5 * u0 * u0) * np.sin(lat) ** 2 / g
    wind = solid_body_wind(p, u0, 0.0, radius)
    return htot - b, wind, b


def williamson_tc6(p, radius=EARTH_RADIUS, omega=OMEGA, g=GRAVITY, w=7.848e-6, K=7.848e-6, R=4, h0=8000.0):
    """Rossby-Haurwitz wave (Williamson TC6).  Returns (h, wind, b)."""
    lon, lat = xyz_to_lonlat(p)
    c, s = np.cos(lat), np.sin(lat)
    u = radius * w * c + radius * K * c ** (R - 1) * (R * s * s - c * c) * np.cos(R * lon)
    v = -radius * K * R * c ** (R - 1) * s * np.sin(R * lon)
    A = 0.5 * w * (2 * omega + w) * c ** 2 + 0.25 * K ** 2 * c ** (2 * R) * (
        (R + 1) * c ** 2 + (2 * R * R - R - 2) - 2 * R * R * c ** (-2.0))
    B = 2 * (omega + w) * K / ((R + 1) * (R + 2)) * c ** R * ((R * R + 2 * R + 2) - (R + 1) ** 2 * c ** 2)
    C = 0.25 * K ** 2 * c ** (2 * R) * ((R + 1) * c ** 2 - (R + 2))
    gh = g * h0 + radius ** 2 * (A + B * np.cos(R * lon) + C * np.cos(2 * R * lon))
    e, n = lonlat_vectors(p)
    wind = u[..., None] * e + v[..., None] * n
    return gh / g, wind, np.zeros_like(gh)


def lima_flag(N: int, squares: int = 8, hot: float = 1000.0, background: float = 1.0) -> np.ndarray:
    """[6, N, N] temperature: checkerboard of `hot` squares on face 0."""
    T = np.full((6, N, N), background, dtype=np.float64)
    k = max(1, N // squares)
    j, i = np.mgrid[0:N, 0:N]
    T[0] = np.where(((i // k) + (j // k)) % 2 == 0, hot, background)
    return T


def gaussian_hill(p, center=(1.0, 0.0, 0.0), width=0.3, amp=1.0):
    c = np.asarray(center, dtype=np.float64)
    c = c / np.linalg.norm(c)
    d2 = np.sum((p - c) ** 2, axis=-1)
    return amp * np.exp(-d2 / (width * width))
