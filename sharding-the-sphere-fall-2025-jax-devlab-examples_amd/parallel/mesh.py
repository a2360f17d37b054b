"""Device mesh and tile sharding: the MI355X counterpart of the reference's
``setup_sharding`` (PY:19-85), ``Mesh(devices, ('tiles',))`` and
``NamedSharding(mesh, P('tiles'))``.

The reference is single-controller (one Python process drives every device,
XLA moves data).  Here the model is SPMD: one process per GPU, rank r drives
``cuda:LOCAL_RANK`` and owns the tiles the partitioner assigns to it; the mesh
object records the global picture identically on every rank.  With
``device_type: cpu`` the ranks are either in-process virtual ranks (the analogue
of ``--xla_force_host_platform_device_count``, PY:64-68) or gloo processes.

Validation and messages follow PY:30-57, except that ``tiles_per_edge > 1`` is
implemented here instead of raising ``NotImplementedError`` (PY:31-37).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

from .partition import num_tiles, partition_report, partition_tiles, tiles_of, validate_device_count


@dataclass
class TileMesh:
    """1-D device mesh along the axis named 'tiles'."""

    devices: List[str]
    axis_names: tuple = ("tiles",)
    device_type: str = "gpu"

    @property
    def size(self) -> int:
        return len(self.devices)

    @property
    def shape(self) -> Dict[str, int]:
        return {self.axis_names[0]: self.size}

    def __repr__(self) -> str:
        return f"TileMesh(devices={self.devices}, axis_names={self.axis_names})"


@dataclass
class TileSharding:
    """Tile -> device assignment (PartitionSpec('tiles') on axis 0, partitioned
    by `strategy`)."""

    mesh: TileMesh
    tiles_per_edge: int
    strategy: str
    owner: List[int] = field(default_factory=list)
    spec: str = "tiles"

    @property
    def num_tiles(self) -> int:
        return len(self.owner)

    def tiles_of(self, device_index: int) -> List[int]:
        return tiles_of(self.owner, device_index)

    def device_of(self, tile: int) -> int:
        return self.owner[tile]

    def __repr__(self) -> str:
        return (f"TileSharding(spec=P({self.spec!r}), strategy={self.strategy!r}, "
                f"num_tiles={self.num_tiles}, devices={self.mesh.size})")


def setup_sharding(config: Dict[str, Any], verbose: bool = True):
    """Validate the parallelization block and build (mesh, sharding).

    ``config`` is the full config dict; reads ``config['parallelization']`` with
    the reference's defaults (PY:21-24).  Returns (TileMesh, TileSharding)."""
    para = config["parallelization"]
    device_type = para.get("device_type", "cpu")
    num_devices = para.get("num_devices", 6)
    tiles_per_edge = para.get("tiles_per_edge", 1)
    strategy = para.get("partition", "auto")
    say = print if verbose else (lambda *a, **k: None)

    say(f"\n{'=' * 70}")
    say("SETTING UP TILE SHARDING (MI355X / RCCL)")
    say(f"{'=' * 70}")
    if not isinstance(tiles_per_edge, int) or tiles_per_edge < 1:
        raise ValueError(f"Error: tiles_per_edge = {tiles_per_edge} must be a positive integer.")
    nt = validate_device_count(num_devices, tiles_per_edge)

    say("  Tile configuration:")
    say(f"    tiles_per_edge: {tiles_per_edge}")
    say(f"    total tiles: {nt} (6 faces × {tiles_per_edge}² tiles/face)")
    say(f"    tiles per device: {nt / num_devices:.1f}")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if device_type == "cpu":
        say("  Device type: CPU (virtual ranks)")
        if world > 1:
            say(f"  gloo process group: {world} ranks")
        else:
            say(f"  In-process virtual ranks: {num_devices}")
        devices = [f"cpu:{i}" for i in range(num_devices)]
        available = num_devices
    else:
        say("  Device type: GPU")
        say(f"  Requested devices: {num_devices}")
        try:
            import torch
            available = torch.cuda.device_count()
        except Exception:
            available = 0
        devices = [f"cuda:{i}" for i in range(num_devices)]
    say(f"  Available devices: {available}")
    say(f"  Using devices: {devices}")

    owner = partition_tiles(tiles_per_edge, num_devices, strategy)
    eff = strategy
    if strategy == "auto":
        eff = "corner" if (tiles_per_edge % 2 == 0 and num_devices in (2, 4, 8)) else "contiguous"
    mesh = TileMesh(devices, ("tiles",), device_type)
    sharding = TileSharding(mesh, tiles_per_edge, eff, owner)
    say(f"  Mesh created: {nt} tiles across {len(devices)} device(s)")
    say(f"  Sharding strategy: PartitionSpec('tiles') on axis 0, {eff} partition")
    if verbose and num_devices > 1:
        say(partition_report(tiles_per_edge, owner))
    if nt > len(devices):
        say("  Note: Multiple tiles per device (one fused launch covers all of a device's tiles)")
    say(f"{'=' * 70}\n")
    return mesh, sharding
