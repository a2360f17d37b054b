"""Reference-compatible halo API (PY:143-246) on (6, N+2, N+2) tensors."""
import numpy as np
import pytest
import torch

from stsphere.models.geometry import CubedSphereGrid
from stsphere.ops.halo import (add_ghosts, exchange_edge_pair, extract_boundary_data, make_halo_exchange,
                               remove_ghosts, set_ghost_data)
from stsphere.parallel.layout import TileLayout
from stsphere.parallel.topology import create_communication_schedule


def _ids(N, ng=1):
    f = torch.arange(6 * N * N, dtype=torch.float64).reshape(6, N, N)
    return add_ghosts(f, ng)


def test_extract_and_set_are_functional():
    N = 5
    fg = _ids(N)
    strip = extract_boundary_data(fg[0], "E", N)
    assert torch.equal(strip, fg[0, 1:N + 1, N])
    new = set_ghost_data(fg[0], "W", strip, N)
    assert torch.equal(new[1:N + 1, 0], strip) and torch.equal(fg[0, 1:N + 1, 0], torch.zeros(N, dtype=fg.dtype))


def test_exchange_edge_pair_reversal():
    N = 4
    fg = _ids(N)
    out = exchange_edge_pair(fg, 0, "N", 1, "N", "R", N)
    assert torch.equal(out[1, N + 1, 1:N + 1], fg[0, N, 1:N + 1].flip(0))
    assert torch.equal(out[0, N + 1, 1:N + 1], fg[1, N, 1:N + 1].flip(0))
    assert torch.equal(fg, _ids(N))          # input untouched (functional)


def test_make_halo_exchange_prints_reference_lines(capsys):
    make_halo_exchange(create_communication_schedule(), 4)
    out = capsys.readouterr().out
    assert "Pre-compiling halo exchange functions..." in out
    assert "  Stage 0: (0,N) ↔ (1,N) [R]" in out
    assert "  Stage 3: (4,S) ↔ (5,W) [T]" in out
    assert out.count("  Stage ") == 12


@pytest.mark.parametrize("ng", [1, 2, 3])
def test_fused_exchange_equals_pairwise_and_geometry(ng):
    N = 6
    sched = create_communication_schedule()
    fg = _ids(N, ng)
    fused = make_halo_exchange(sched, N, ng=ng, verbose=False)(fg)
    pair = fg
    for st in sched:
        for (fa, ea), (fb, eb), op in st:
            pair = exchange_edge_pair(pair, fa, ea, fb, eb, op, N)
    assert torch.equal(fused, pair)
    # ghost strips hold the geometric neighbour ids (from the tile layout's map)
    L = TileLayout(N, 1, 1, ng=ng)
    src = L.ghost_sources(0)          # [6,4,ng,N] global ids
    P = N + 2 * ng
    for f in range(6):
        for k in range(ng):
            assert torch.equal(fused[f, ng:ng + N, ng - 1 - k].long(), torch.as_tensor(src[f, 0, k]))
            assert torch.equal(fused[f, ng:ng + N, ng + N + k].long(), torch.as_tensor(src[f, 1, k]))
            assert torch.equal(fused[f, ng - 1 - k, ng:ng + N].long(), torch.as_tensor(src[f, 2, k]))
            assert torch.equal(fused[f, ng + N + k, ng:ng + N].long(), torch.as_tensor(src[f, 3, k]))
    # corners untouched (the reference never fills them)
    assert (fused[:, :ng, :ng] == 0).all() and (fused[:, -ng:, -ng:] == 0).all()
    assert torch.equal(remove_ghosts(fused, N), remove_ghosts(fg, N))


def test_batched_fields():
    N = 4
    fg = torch.stack([_ids(N), 2 * _ids(N)])
    out = make_halo_exchange(create_communication_schedule(), N, verbose=False)(fg)
    assert torch.equal(out[1], 2 * out[0])


def test_bad_schedule_rejected():
    bad = ((((0, "N"), (2, "N"), "R"),),)
    with pytest.raises(ValueError, match="not a cube edge"):
        make_halo_exchange(bad, 4, verbose=False)
