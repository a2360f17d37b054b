"""Multi-rank paths without a cluster: in-process virtual ranks and
multi-process gloo (modes (a) and (b))."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from stsphere.engine import Engine, VirtualCluster
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.models.advection import Advection
from stsphere.parallel.layout import TileLayout


@pytest.mark.parametrize("t,R", [(1, 2), (1, 3), (1, 6), (2, 4), (2, 8), (2, 12)])
def test_virtual_ranks_bitwise_equal_single(t, R):
    N = 12
    g = CubedSphereGrid(N)
    single = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g)
    vc = VirtualCluster(lambda: ShallowWater("tc5"), TileLayout(N, t, R, ng=2), grid=g, dt=single.dt)
    single.step(3)
    vc.step(3)
    for f in range(4):
        assert np.array_equal(single.global_field(f), vc.global_field(f))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, t, staged, outdir):
    import torch.distributed as dist
    from stsphere.parallel.comm import TorchDistTransport
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = TileLayout(N, t, world, ng=2)
        phys = ShallowWater("tc5")
        tr = TorchDistTransport(L.plan(rank), 4, torch.float64, torch.device("cpu"), staged=staged)
        e = Engine(phys, L, rank, transport=tr, dt=300.0)
        e.step(3)
        np.save(os.path.join(outdir, f"r{rank}.npy"), e.tiles_view().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,t,staged", [(2, 1, False), (3, 1, True), (4, 2, False), (6, 1, False), (6, 1, True),
                                            (8, 2, False), (8, 2, True)])
def test_gloo_multiprocess_equals_single(world, t, staged):
    N = 8
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), N, t, staged, out), nprocs=world, join=True)
    L = TileLayout(N, t, world, ng=2)
    g = CubedSphereGrid(N)
    single = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g, dt=300.0)
    single.step(3)
    from stsphere.engine import assemble_global
    for f in range(4):
        glob = assemble_global(L, {r: np.load(os.path.join(out, f"r{r}.npy"))[f] for r in range(world)})
        assert np.array_equal(glob, single.global_field(f))


def test_loopback_layout_equals_single():
    from stsphere.parallel.comm import LoopbackTransport
    N = 12
    g = CubedSphereGrid(N)
    L = TileLayout(N, 2, 1, ng=2, loopback=True)
    p = L.plan(0)
    assert p.recv_peers == [0] and p.send_peers == [0] and (p.ghost_map < 0).all() and (p.push_map < 0).all()
    single = Engine(ShallowWater("tc5"), TileLayout(N, 2, 1, ng=2), grid=g)
    lb = Engine(ShallowWater("tc5"), L, grid=g, dt=single.dt,
                transport=LoopbackTransport(p, 4, torch.float64, torch.device("cpu")))
    single.step(3)
    lb.step(3)
    assert torch.equal(single.tiles_view(), lb.tiles_view())
