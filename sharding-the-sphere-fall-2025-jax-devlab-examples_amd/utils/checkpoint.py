"""Checkpoint / restart (PDF s.4 "Checkpoint/restart (Orbax)", s.6 "Restarts").

Orbax-like directory layout, independent of the GPU count and tiling that
wrote it:

    <root>/<step:08d>/
        _METADATA                 JSON: step, time, dt, grid, fields, dtype, integrator,
                                  writer tiling (tiles_per_edge, owner map), config
        state/                    zarr v2 group
            <field>/              shape (6, N, N), chunks (1, n, n): one chunk per tile
        _CHECKPOINT_COMPLETE      commit marker, written last

Every rank writes exactly the chunks of the tiles it owns (no gather); a
restore with any tiling / rank count reads the global arrays back.  A
checkpoint without the commit marker is ignored by ``latest_checkpoint``.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Any, Dict, Iterable, List, Optional

import numpy as np

from . import zarr_lite

COMMIT = "_CHECKPOINT_COMPLETE"
META = "_METADATA"


def step_dir(root: str, step: int) -> str:
    return os.path.join(root, f"{int(step):08d}")


def begin(root: str, step: int, meta: Dict[str, Any], fields: List[str], N: int, n: int, dtype) -> str:
    """Rank 0: create the step directory, metadata and empty arrays."""
    d = step_dir(root, step)
    if os.path.exists(d):
        shutil.rmtree(d)
    os.makedirs(d)
    with open(os.path.join(d, META), "w") as f:
        json.dump(meta, f, indent=2, default=str)
    g = zarr_lite.create_group(os.path.join(d, "state"), attrs={"fields": fields, "N": N, "tile": n})
    for name in fields:
        zarr_lite.create_array(g, name, (6, N, N), np.dtype(dtype), chunks=(1, n, n))
    return d


def write_tiles(d: str, fields: List[str], tiles: Iterable[int], tile_origin, values: np.ndarray, n: int) -> None:
    """Write this rank's tiles.  values: [F, T_local, n, n]; tile_origin(tid) ->
    (face, I0, J0)."""
    g = os.path.join(d, "state")
    for li, tid in enumerate(tiles):
        f, I0, J0 = tile_origin(tid)
        for k, name in enumerate(fields):
            zarr_lite.write_chunk(g, name, (f, J0 // n, I0 // n), values[k, li][None])


def commit(d: str) -> None:
    with open(os.path.join(d, COMMIT), "w") as f:
        f.write(str(time.time()))


def is_complete(d: str) -> bool:
    return os.path.exists(os.path.join(d, COMMIT))


def list_checkpoints(root: str) -> List[int]:
    if not os.path.isdir(root):
        return []
    out = []
    for e in os.listdir(root):
        if e.isdigit() and is_complete(os.path.join(root, e)):
            out.append(int(e))
    return sorted(out)


def latest_checkpoint(root: str) -> Optional[str]:
    steps = list_checkpoints(root)
    return step_dir(root, steps[-1]) if steps else None


def read_meta(d: str) -> Dict[str, Any]:
    with open(os.path.join(d, META)) as f:
        return json.load(f)


def read_fields(d: str, fields: Optional[List[str]] = None) -> Dict[str, np.ndarray]:
    """Global arrays (6, N, N) of a committed checkpoint."""
    if not is_complete(d):
        raise FileNotFoundError(f"checkpoint {d} is incomplete (no {COMMIT})")
    g = os.path.join(d, "state")
    names = fields or zarr_lite.read_attrs(g)["fields"]
    return {k: zarr_lite.read_array(g, k) for k in names}


def prune(root: str, keep: int) -> None:
    steps = list_checkpoints(root)
    for s in steps[:-keep] if keep > 0 else []:
        shutil.rmtree(step_dir(root, s), ignore_errors=True)
