"""Tile partitioner and the reference's device-count validation (PY:30-57)."""
import pytest

from stsphere.parallel import partition as P
from stsphere.parallel.mesh import setup_sharding


def test_valid_counts():
    assert P.valid_device_counts(1) == [1, 2, 3, 6]
    assert P.valid_device_counts(2) == [1, 2, 3, 4, 6, 8, 12, 24]


def test_errors_match_reference_text():
    with pytest.raises(ValueError, match="exceeds num_tiles = 6"):
        P.validate_device_count(7, 1)
    with pytest.raises(ValueError, match=r"valid device counts are:\n  \[1, 2, 3, 6\]"):
        P.validate_device_count(4, 1)


@pytest.mark.parametrize("nd,cut", [(1, 0), (2, 8), (4, 16), (8, 24)])
def test_corner_partition_cuts(nd, cut):
    owner = P.partition_tiles(2, nd, "corner")
    assert P.cut_edges(2, owner) == cut
    assert len(set(P.balance(owner))) == 1


def test_corner_8_is_cube_graph():
    owner = P.partition_tiles(2, 8, "corner")
    g = P.device_graph(2, owner)
    assert len(g) == 12 and set(g.values()) == {2}
    deg = [sum(1 for e in g if d in e) for d in range(8)]
    assert deg == [3] * 8


def test_contiguous_is_reference_block_split():
    owner = P.partition_tiles(1, 3, "contiguous")
    assert owner == [0, 0, 1, 1, 2, 2]
    assert P.cut_edges(2, P.partition_tiles(2, 8, "contiguous")) == 36


def test_tile_adjacency_regular():
    for t in (1, 2, 3):
        adj = P.tile_adjacency(t)
        assert len(adj) == 12 * t * t
        deg = {}
        for a, b in adj:
            deg[a] = deg.get(a, 0) + 1
            deg[b] = deg.get(b, 0) + 1
        assert set(deg.values()) == {4}


def test_setup_sharding_banner(capsys):
    mesh, sh = setup_sharding({"parallelization": {"tiles_per_edge": 2, "num_devices": 8, "device_type": "cpu"}})
    out = capsys.readouterr().out
    assert "total tiles: 24 (6 faces × 2² tiles/face)" in out
    assert "tiles per device: 3.0" in out
    assert mesh.axis_names == ("tiles",) and mesh.size == 8
    assert sh.strategy == "corner" and sorted(sh.tiles_of(0)) == sh.tiles_of(0) and len(sh.tiles_of(0)) == 3
    with pytest.raises(ValueError):
        setup_sharding({"parallelization": {"tiles_per_edge": 1, "num_devices": 4}}, verbose=False)
    # reference defaults (PY:21-24): cpu, 6 devices, tiles_per_edge 1
    mesh, sh = setup_sharding({"parallelization": {}}, verbose=False)
    assert mesh.size == 6 and sh.num_tiles == 6 and mesh.device_type == "cpu"
