"""Analysis / visualisation products (PDF s.6 "Analysis/Viz"; figures on
s.4, s.12, s.13, s.17, s.18).

* ``sphere_plot``   3-D view of a [6, N, N] field on the sphere, optional log
                    colour scale (Lima-flag diffusion, PDF s.12 / s.17)
* ``latlon_band``   longitude-latitude scatter of a band, e.g. 0-360 x +-50 deg
                    (cosine bell, PDF s.13)
* ``six_panel``     per-face images of an initial and a final field
                    (PDF s.18 "Initial vs Final")
* ``mesh_plot``     the cubed-sphere dual mesh outline (PDF s.4)

Headless (Agg backend); every function writes a PNG and returns its path.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from ..models.geometry import CubedSphereGrid


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def sphere_plot(field: np.ndarray, grid: CubedSphereGrid, path: str, title: str = "", log: bool = False,
                cmap: str = "inferno", elev: float = 25.0, azim: float = -60.0) -> str:
    plt = _plt()
    from matplotlib.colors import LogNorm, Normalize
    c = grid.centers().reshape(-1, 3)
    v = np.asarray(field).reshape(-1)
    norm = LogNorm(vmin=max(v[v > 0].min() if (v > 0).any() else 1e-12, 1e-12), vmax=v.max()) if log else \
        Normalize(vmin=v.min(), vmax=v.max())
    fig = plt.figure(figsize=(7, 6))
    ax = fig.add_subplot(111, projection="3d")
    sc = ax.scatter(c[:, 0], c[:, 1], c[:, 2], c=v, cmap=cmap, norm=norm, s=max(1.0, 4000.0 / grid.N ** 2 * 6),
                    marker="s", linewidths=0)
    ax.view_init(elev=elev, azim=azim)
    ax.set_box_aspect((1, 1, 1))
    ax.set_axis_off()
    fig.colorbar(sc, ax=ax, shrink=0.7)
    ax.set_title(title)
    fig.savefig(path, dpi=110, bbox_inches="tight")
    plt.close(fig)
    return path


def latlon_band(field: np.ndarray, grid: CubedSphereGrid, path: str, lat_max_deg: float = 50.0, title: str = "",
                cmap: str = "viridis") -> str:
    plt = _plt()
    lon, lat = grid.lonlat()
    lon, lat = np.degrees(lon).reshape(-1), np.degrees(lat).reshape(-1)
    v = np.asarray(field).reshape(-1)
    m = np.abs(lat) <= lat_max_deg
    fig, ax = plt.subplots(figsize=(10, 3.2))
    sc = ax.scatter(lon[m], lat[m], c=v[m], cmap=cmap, s=6, marker="s", linewidths=0)
    ax.set_xlim(0, 360)
    ax.set_ylim(-lat_max_deg, lat_max_deg)
    ax.set_xlabel("longitude (deg E)")
    ax.set_ylabel("latitude (deg)")
    ax.set_title(title or f"peak {v.max():.1f}")
    fig.colorbar(sc, ax=ax)
    fig.savefig(path, dpi=110, bbox_inches="tight")
    plt.close(fig)
    return path


def six_panel(initial: np.ndarray, final: np.ndarray, path: str, title: str = "Initial vs Final",
              cmap: str = "viridis") -> str:
    plt = _plt()
    vmin = min(initial.min(), final.min())
    vmax = max(initial.max(), final.max())
    fig, axes = plt.subplots(2, 6, figsize=(15, 5.2))
    for row, (name, f) in enumerate((("initial", initial), ("final", final))):
        for face in range(6):
            ax = axes[row, face]
            im = ax.imshow(f[face], origin="lower", cmap=cmap, vmin=vmin, vmax=vmax)
            ax.set_title(f"{name} face {face}", fontsize=9)
            ax.set_xticks([])
            ax.set_yticks([])
    fig.colorbar(im, ax=axes.ravel().tolist(), shrink=0.8)
    fig.suptitle(title)
    fig.savefig(path, dpi=100, bbox_inches="tight")
    plt.close(fig)
    return path


def mesh_plot(grid: CubedSphereGrid, path: str, stride: int = 1) -> str:
    plt = _plt()
    v = grid.vertices()
    fig = plt.figure(figsize=(6, 6))
    ax = fig.add_subplot(111, projection="3d")
    for f in range(6):
        for j in range(0, grid.N + 1, stride):
            ax.plot(v[f, j, :, 0], v[f, j, :, 1], v[f, j, :, 2], lw=0.4, color="k")
        for i in range(0, grid.N + 1, stride):
            ax.plot(v[f, :, i, 0], v[f, :, i, 1], v[f, :, i, 2], lw=0.4, color="k")
    ax.set_box_aspect((1, 1, 1))
    ax.set_axis_off()
    ax.set_title(f"Cube sphere mesh (Ne={grid.N}x{grid.N}, {6 * grid.N * grid.N} quads)")
    fig.savefig(path, dpi=110, bbox_inches="tight")
    plt.close(fig)
    return path


def history_frames(history_path: str, field: str, grid: CubedSphereGrid, outdir: str, log: bool = False,
                   every: int = 1) -> Sequence[str]:
    """Render a zarr history (utils.history) to one sphere PNG per frame."""
    import os
    from .history import read_history
    from . import zarr_lite
    h = read_history(history_path, field)
    t = zarr_lite.read_array(history_path, "time")
    os.makedirs(outdir, exist_ok=True)
    out = []
    for k in range(0, h.shape[0], every):
        out.append(sphere_plot(h[k], grid, os.path.join(outdir, f"{field}_{k:04d}.png"),
                               title=f"{field}  day {t[k] / 86400.0:.2f}", log=log))
    return out


def history_products(history_path: str, field: str, outdir: str, grid: Optional[CubedSphereGrid] = None,
                     log: bool = False, every: int = 1,
                     products: Sequence[str] = ("frames", "band", "six")) -> Sequence[str]:
    """The analysis products of a run from its zarr history (PDF s.6
    "Analysis/Viz: jax.zarr"):

    * ``frames``  one 3-D sphere PNG per history frame (PDF s.12 / s.17);
    * ``band``    lon-lat equatorial band (0-360 x +-50 deg) of the first and
                  the last frame (PDF s.13 "Cosine Bell Advection - Equatorial
                  Band", title carries day and peak);
    * ``six``     per-face initial vs final panels (PDF s.18).
    """
    import os
    from .history import read_history
    from . import zarr_lite
    if grid is None:
        grid = CubedSphereGrid(int(zarr_lite.read_attrs(history_path)["N"]))
    h = read_history(history_path, field)
    t = zarr_lite.read_array(history_path, "time")
    os.makedirs(outdir, exist_ok=True)
    out = []
    if "frames" in products:
        out += list(history_frames(history_path, field, grid, os.path.join(outdir, "frames"), log=log, every=every))
    last = h.shape[0] - 1
    if "band" in products:
        for k, name in ((0, "initial"), (last, "final")):
            out.append(latlon_band(h[k], grid, os.path.join(outdir, f"{field}_band_{name}.png"),
                                   title=f"{field} equatorial band, day {t[k] / 86400.0:.2f}, peak {h[k].max():.1f}"))
    if "six" in products:
        out.append(six_panel(h[0], h[last], os.path.join(outdir, f"{field}_six_panel.png"),
                             title=f"{field}: initial (day {t[0] / 86400.0:.2f}) vs final (day {t[last] / 86400.0:.2f})"))
    return out
