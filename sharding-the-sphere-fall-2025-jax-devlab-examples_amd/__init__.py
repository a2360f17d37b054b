"""stsphere: an MI355X-native cubed-sphere finite-volume framework with the
capabilities of the "Sharding the Sphere" JAX DevLab examples (diffusion,
tracer advection, shallow water on a 6-panel cubed sphere, tile sharding,
12-edge halo exchange, zarr history, Orbax-style restarts).

Import as ``stsphere`` (the source directory name is not an identifier).
"""
__version__ = "0.1.0"

from .parallel.topology import (EDGES, FACE_FRAMES, LINKS, apply_operations, create_communication_schedule,
                                derive_edge_pairs, edge_coloring, neighbor_cell)
from .parallel.partition import num_tiles, partition_tiles, valid_device_counts, validate_device_count
from .parallel.layout import TileLayout, RankPlan
from .parallel.mesh import TileMesh, TileSharding, setup_sharding
from .utils.config import Config, load_config, save_config
from .models.geometry import CubedSphereGrid
from .models.integrators import get_integrator
from .models.swe import ShallowWater
from .models.advection import Advection
from .models.diffusion import Diffusion
from .ops.halo import (exchange_edge_pair, extract_boundary_data, make_halo_exchange, set_ghost_data,
                       remove_ghosts, add_ghosts)
from .engine import Engine, GraphStepper, VirtualCluster
from .driver import Solver, make_physics
from .ensemble import Ensemble

__all__ = [
    "apply_operations", "create_communication_schedule", "derive_edge_pairs", "edge_coloring", "neighbor_cell",
    "num_tiles", "partition_tiles", "valid_device_counts", "validate_device_count", "TileLayout", "RankPlan",
    "TileMesh", "TileSharding", "setup_sharding", "Config", "load_config", "save_config", "CubedSphereGrid",
    "get_integrator", "ShallowWater", "Advection", "Diffusion", "exchange_edge_pair", "extract_boundary_data",
    "make_halo_exchange", "set_ghost_data", "remove_ghosts", "add_ghosts", "Engine", "GraphStepper",
    "VirtualCluster", "Solver", "make_physics", "Ensemble",
]
