"""Minimal Zarr v2 store (directory layout, no compression) in NumPy.

The reference's pipeline writes geometry, initial conditions, history and
analysis products through zarr (PDF s.6 img: "jax.zarr").  The zarr package is
not installed here, so this module writes the v2 on-disk format directly:

    <group>/.zgroup                {"zarr_format": 2}
    <group>/.zattrs                JSON attributes
    <group>/<array>/.zarray        shape / chunks / dtype / order / compressor=null
    <group>/<array>/.zattrs
    <group>/<array>/<i>.<j>...     raw little-endian C-order chunk bytes

Files written here open with ``zarr.open(path)`` in a standard zarr-python.
Chunks are written independently, so several ranks can each write the chunks
of the tiles they own (partition-independent restarts).
Edge chunks are stored full-size (zero padded), as the zarr spec requires.
"""
from __future__ import annotations

import itertools
import json
import os
from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np


def _dump(path: str, obj: Dict[str, Any]) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=2, sort_keys=True, default=_json_default)
    os.replace(tmp, path)


def _json_default(o):
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise TypeError(type(o))


def create_group(path: str, attrs: Optional[Dict[str, Any]] = None) -> str:
    os.makedirs(path, exist_ok=True)
    _dump(os.path.join(path, ".zgroup"), {"zarr_format": 2})
    if attrs is not None:
        _dump(os.path.join(path, ".zattrs"), attrs)
    return path


def read_attrs(path: str) -> Dict[str, Any]:
    p = os.path.join(path, ".zattrs")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def write_attrs(path: str, attrs: Dict[str, Any]) -> None:
    _dump(os.path.join(path, ".zattrs"), attrs)


def create_array(group: str, name: str, shape: Sequence[int], dtype, chunks: Optional[Sequence[int]] = None,
                 attrs: Optional[Dict[str, Any]] = None, fill_value=0) -> str:
    dtype = np.dtype(dtype)
    shape = tuple(int(s) for s in shape)
    chunks = tuple(int(c) for c in (chunks or shape))
    apath = os.path.join(group, name)
    os.makedirs(apath, exist_ok=True)
    meta = {
        "zarr_format": 2,
        "shape": list(shape),
        "chunks": list(chunks),
        "dtype": dtype.newbyteorder("<").str if dtype.byteorder not in ("|",) else dtype.str,
        "compressor": None,
        "fill_value": fill_value,
        "order": "C",
        "filters": None,
        "dimension_separator": ".",
    }
    _dump(os.path.join(apath, ".zarray"), meta)
    _dump(os.path.join(apath, ".zattrs"), attrs or {})
    return apath


def array_meta(group: str, name: str) -> Dict[str, Any]:
    with open(os.path.join(group, name, ".zarray")) as f:
        return json.load(f)


def _chunk_key(idx: Sequence[int]) -> str:
    return ".".join(str(int(i)) for i in idx) if len(idx) else "0"


def write_chunk(group: str, name: str, chunk_idx: Sequence[int], data: np.ndarray,
                meta: Optional[Dict[str, Any]] = None) -> None:
    """Write one chunk (atomic rename).  ``meta``: the array's metadata when the
    caller holds it (a writer of many chunks skips re-reading .zarray)."""
    meta = meta or array_meta(group, name)
    chunks = tuple(meta["chunks"])
    dt = np.dtype(meta["dtype"])
    data = np.asarray(data)
    if data.shape == chunks and data.dtype == dt:
        buf = data
    else:
        buf = np.zeros(chunks, dtype=dt)
        sl = tuple(slice(0, s) for s in data.shape)
        buf[sl] = data
    p = os.path.join(group, name, _chunk_key(chunk_idx))
    tmp = p + ".tmp"
    with open(tmp, "wb") as f:
        f.write(np.ascontiguousarray(buf).tobytes())
    os.replace(tmp, p)


def write_region(group: str, name: str, start: Sequence[int], data: np.ndarray) -> None:
    """Write `data` whose origin is chunk-aligned at `start` and which covers
    whole chunks (or ends at the array edge)."""
    meta = array_meta(group, name)
    chunks = meta["chunks"]
    shape = meta["shape"]
    data = np.asarray(data)
    for s, c in zip(start, chunks):
        if s % c:
            raise ValueError("region start must be chunk aligned")
    ranges = [range(s // c, (s + d + c - 1) // c) for s, d, c in zip(start, data.shape, chunks)]
    for idx in itertools.product(*ranges):
        lo = [i * c - s for i, c, s in zip(idx, chunks, start)]
        hi = [min(l + c, d, sh - s) for l, c, d, sh, s in zip(lo, chunks, data.shape, shape, start)]
        write_chunk(group, name, idx, data[tuple(slice(l, h) for l, h in zip(lo, hi))])


def write_array(group: str, name: str, data: np.ndarray, chunks: Optional[Sequence[int]] = None,
                attrs: Optional[Dict[str, Any]] = None) -> None:
    data = np.asarray(data)
    create_array(group, name, data.shape, data.dtype, chunks, attrs)
    write_region(group, name, (0,) * data.ndim, data)


def read_array(group: str, name: str) -> np.ndarray:
    meta = array_meta(group, name)
    shape, chunks = tuple(meta["shape"]), tuple(meta["chunks"])
    if meta.get("compressor") is not None:
        raise ValueError("compressed zarr arrays are not supported by zarr_lite")
    dt = np.dtype(meta["dtype"])
    out = np.full(shape, meta.get("fill_value") or 0, dtype=dt)
    sep = meta.get("dimension_separator", ".")
    nchunks = [(s + c - 1) // c for s, c in zip(shape, chunks)]
    for idx in itertools.product(*[range(n) for n in nchunks]):
        key = sep.join(str(i) for i in idx) if idx else "0"
        p = os.path.join(group, name, key)
        if not os.path.exists(p):
            continue
        buf = np.fromfile(p, dtype=dt).reshape(chunks)
        lo = [i * c for i, c in zip(idx, chunks)]
        hi = [min(l + c, s) for l, c, s in zip(lo, chunks, shape)]
        out[tuple(slice(l, h) for l, h in zip(lo, hi))] = buf[tuple(slice(0, h - l) for l, h in zip(lo, hi))]
    return out


def read_chunk(group: str, name: str, chunk_idx: Sequence[int]) -> np.ndarray:
    meta = array_meta(group, name)
    dt = np.dtype(meta["dtype"])
    p = os.path.join(group, name, _chunk_key(chunk_idx))
    return np.fromfile(p, dtype=dt).reshape(tuple(meta["chunks"]))


def list_arrays(group: str):
    return sorted(d for d in os.listdir(group) if os.path.exists(os.path.join(group, d, ".zarray")))


def resize_first_axis(group: str, name: str, new_len: int) -> None:
    """Grow an append-axis (history time axis)."""
    meta = array_meta(group, name)
    meta["shape"][0] = int(new_len)
    _dump(os.path.join(group, name, ".zarray"), meta)
