"""History output (PDF s.6 "History: jax.zarr") and JSONL metrics.

History: one zarr v2 group per run,

    history.zarr/<field>   shape (n_out, 6, N, N), chunks (1, 1, n, n)
    history.zarr/time      shape (n_out,)  seconds
    history.zarr/step      shape (n_out,)

written tile-chunk by tile-chunk by the owning ranks (no gather).
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, List, Optional

import numpy as np

from . import zarr_lite


class HistoryWriter:
    def __init__(self, path: str, fields: List[str], N: int, n: int, n_out: int, dtype=np.float64,
                 attrs: Optional[Dict[str, Any]] = None, create: bool = True, frame_chunks: bool = False):
        """Chunks of one tile per field and frame (every rank writes its own
        tiles), or ``frame_chunks``: one whole [6, N, N] field per chunk, for a
        writer that holds every tile (one file per field and frame instead of
        one per tile: ~10 ms -> ~1 ms per C96 t = 2 frame)."""
        self.path = path
        self.fields = fields
        self.N, self.n, self.n_out = N, n, n_out
        self.count = 0
        if create:
            zarr_lite.create_group(path, attrs=dict(attrs or {}, fields=fields, N=N))
            ch = (1, 6, N, N) if frame_chunks else (1, 1, n, n)
            for f in fields:
                zarr_lite.create_array(path, f, (n_out, 6, N, N), np.dtype(dtype), chunks=ch)
            zarr_lite.create_array(path, "time", (n_out,), np.float64, chunks=(n_out,))
            zarr_lite.create_array(path, "step", (n_out,), np.int64, chunks=(n_out,))
        self._meta = {f: zarr_lite.array_meta(path, f) for f in fields + ["time", "step"]}
        self.frame_chunks = tuple(self._meta[fields[0]]["chunks"])[1] == 6 if fields else False
        self._times = np.zeros(n_out)
        self._steps = np.zeros(n_out, dtype=np.int64)

    def write_tiles(self, k: int, tiles, tile_origin, values: np.ndarray) -> None:
        """values [F, T_local, n, n] for history slot k (with frame chunks:
        every tile of the grid)."""
        if k >= self.n_out:
            return
        n, N = self.n, self.N
        if self.frame_chunks:
            frame = np.zeros((len(self.fields), 6, N, N), dtype=np.dtype(self._meta[self.fields[0]]["dtype"]))
            seen = 0
            for li, tid in enumerate(tiles):
                f, I0, J0 = tile_origin(tid)
                frame[:, f, J0:J0 + n, I0:I0 + n] = values[:, li]
                seen += 1
            if seen * n * n != 6 * N * N:
                raise ValueError("a frame-chunked history is written whole (every tile in one call)")
            for j, name in enumerate(self.fields):
                zarr_lite.write_chunk(self.path, name, (k, 0, 0, 0), frame[j][None], meta=self._meta[name])
            return
        for li, tid in enumerate(tiles):
            f, I0, J0 = tile_origin(tid)
            for j, name in enumerate(self.fields):
                zarr_lite.write_chunk(self.path, name, (k, f, J0 // n, I0 // n), values[j, li][None, None],
                                      meta=self._meta[name])

    def write_time(self, k: int, t: float, step: int) -> None:
        if k >= self.n_out:
            return
        self._times[k] = t
        self._steps[k] = step
        zarr_lite.write_chunk(self.path, "time", (0,), self._times, meta=self._meta["time"])
        zarr_lite.write_chunk(self.path, "step", (0,), self._steps, meta=self._meta["step"])


def read_history(path: str, field: str) -> np.ndarray:
    return zarr_lite.read_array(path, field)


class MetricsLogger:
    """Per-step JSONL metrics (rank 0)."""

    def __init__(self, path: Optional[str], enabled: bool = True):
        self.path = path
        self.enabled = enabled and path is not None
        self.t0 = time.perf_counter()
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def log(self, **rec) -> Dict[str, Any]:
        rec.setdefault("wall_s", time.perf_counter() - self.t0)
        if self.enabled:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
        return rec


def read_metrics(path: str) -> List[Dict[str, Any]]:
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]
