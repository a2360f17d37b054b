"""Direct xGMI halo exchange (ops/xgmi.py + XG stage kernels) on an MI355X.

* Loopback: one rank whose every ghost goes through the ring (the rank is its
  own peer).  This exercises the push encoding, the counters, the polls and
  the ring rotation in one process.
* Two processes sharing one GPU, ranks 0 and 1 of a 2-rank layout.  The rings
  are mapped across processes with dmabuf IPC, and the two ranks' kernels run
  concurrently and hand ghosts to each other.  This is the multi-GPU protocol
  minus the xGMI wire.

Both must match the single-rank run bit for bit (fp64).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from stsphere.engine import Engine, assemble_global
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.models.advection import Advection
from stsphere.parallel.comm import NativeBuffers
from stsphere.parallel.layout import TileLayout

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("N,t,integ,use_graph", [(24, 2, "ssprk3", True), (24, 2, "ssprk3", False),
                                                 (32, 2, "rk4", True), (20, 1, "euler", True),
                                                 (48, 2, "ssprk2", True)])
def test_xgmi_loopback_matches_single(N, t, integ, use_graph):
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.ops.xgmi import XgmiHalo
    g = CubedSphereGrid(N)
    a = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g, device="cuda", backend="hip", integrator=integ)
    L = TileLayout(N, t, 1, ng=2, loopback=True)
    b = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", integrator=integ, dt=a.dt,
               transport=NativeBuffers(L.plan(0), 4, torch.float64, torch.device("cuda")))
    xg = XgmiHalo(b, timeout_s=1.0)
    ns = NativeStepper(b, use_graph=use_graph, steps_per_graph=4, xgmi=xg)
    a.step(12)
    ns.run(12)
    torch.cuda.synchronize()
    ns.check()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    # epochs only grow; the runner's warm-up period on a scratch copy counts too
    assert int(xg.epoch.min()) == int(xg.epoch.max()) >= 12 * len(b.integ.stages)
    ns.close()
    xg.close()


def test_xgmi_loopback_advection_and_reprime():
    """Tracer advection (F = 1) plus a state reset mid-run (re-delivery)."""
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.ops.xgmi import XgmiHalo
    N = 32
    g = CubedSphereGrid(N)
    a = Engine(Advection(), TileLayout(N, 2, 1, ng=2), grid=g, device="cuda", backend="hip")
    L = TileLayout(N, 2, 1, ng=2, loopback=True)
    b = Engine(Advection(), L, grid=g, device="cuda", backend="hip", dt=a.dt,
               transport=NativeBuffers(L.plan(0), 1, torch.float64, torch.device("cuda")))
    xg = XgmiHalo(b, timeout_s=1.0)
    ns = NativeStepper(b, use_graph=True, steps_per_graph=5, xgmi=xg)
    a.step(5)
    ns.run(5)
    torch.cuda.synchronize()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    q0 = torch.as_tensor(a.physics.initial_state(a.geo), dtype=torch.float64)
    a.set_state(q0)
    b.set_state(q0)
    xg.prime()
    a.step(5)
    ns.run(5)
    torch.cuda.synchronize()
    ns.check()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    ns.close()
    xg.close()


@pytest.mark.parametrize("N,t,dtype", [(24, 2, torch.float64), (48, 1, torch.float64), (32, 2, torch.float32)])
def test_xgmi_loopback_march_matches_single(N, t, dtype):
    """The streaming stage (march_kernel.hip, 64 x 4) with the direct xGMI
    exchange: every ghost of a loopback rank is read from its own ring by the
    march's halo lanes and edge rows and stored into it by the cells that feed
    it (tagged granules), against the one-rank march: bit for bit."""
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.ops.xgmi import XgmiHalo
    g = CubedSphereGrid(N)
    a = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g, device="cuda", backend="hip", dtype=dtype,
               block=(64, 4))
    L = TileLayout(N, t, 1, ng=2, loopback=True)
    b = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", dtype=dtype, dt=a.dt, block=(64, 4),
               transport=NativeBuffers(L.plan(0), 4, dtype, torch.device("cuda")))
    assert a.compute.march and b.compute.march
    xg = XgmiHalo(b, timeout_s=1.0)
    ns = NativeStepper(b, use_graph=True, steps_per_graph=4, xgmi=xg)
    a.step(8)
    ns.run(8)
    torch.cuda.synchronize()
    ns.check()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert int(xg.epoch.min()) == int(xg.epoch.max()) >= 8 * len(b.integ.stages)
    ns.close()
    xg.close()


def _worker(rank, world, port, N, t, steps, outdir, block=None, rounds=1):
    import ctypes
    import torch.distributed as dist
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.ops.xgmi import XgmiHalo
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = TileLayout(N, t, world, ng=2)
        dev = torch.device("cuda:0")
        held = []
        for _ in range(rounds):
            # rounds > 1: the next exchange reuses this process's pooled ring
            # and the peers open its IPC handle again
            e = Engine(ShallowWater("tc5"), L, rank, device=dev, backend="hip", dt=200.0, block=block,
                       transport=NativeBuffers(L.plan(rank), 4, torch.float64, dev))
            xg = XgmiHalo(e, timeout_s=5.0)
            ns = NativeStepper(e, use_graph=True, steps_per_graph=5, xgmi=xg)
            ns.run(steps)
            torch.cuda.synchronize()
            ns.check()
            np.save(os.path.join(outdir, f"r{rank}.npy"), e.tiles_view().cpu().numpy())
            dist.barrier()
            ns.close()
            xg.close()
            st = (ctypes.c_longlong * 4)()
            xg._lib.stsp_xg_pool(st)
            held.append(int(st[0]))
            dist.barrier()
        assert len(set(held)) == 1, held          # no new ring after the first round
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,t", [(2, 2), (4, 2), (3, 1)])
def test_xgmi_multiprocess_one_gpu(world, t):
    N, steps = 24, 10
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), N, t, steps, out), nprocs=world, join=True)
    g = CubedSphereGrid(N)
    single = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g, device="cuda", backend="hip", dt=200.0)
    single.step(steps)
    L = TileLayout(N, t, world, ng=2)
    for f in range(4):
        glob = assemble_global(L, {r: np.load(os.path.join(out, f"r{r}.npy"))[f] for r in range(world)})
        assert np.array_equal(glob, single.global_field(f)), f


def test_xgmi_multiprocess_rings_reused():
    """Two exchanges one after the other in the same two processes: the second
    runs on the pooled rings (peers reopen the same IPC handles) and still
    equals the one-rank run bit for bit."""
    N, t, world, steps = 24, 2, 2, 6
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), N, t, steps, out, None, 2), nprocs=world, join=True)
    g = CubedSphereGrid(N)
    single = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g, device="cuda", backend="hip", dt=200.0)
    single.step(steps)
    L = TileLayout(N, t, world, ng=2)
    for f in range(4):
        glob = assemble_global(L, {r: np.load(os.path.join(out, f"r{r}.npy"))[f] for r in range(world)})
        assert np.array_equal(glob, single.global_field(f)), f


def test_xgmi_multiprocess_one_gpu_march():
    """Two processes sharing one GPU, both marching (64 x 4): each rank's remote
    ghosts arrive through the other's stores into its ring; the assembled state
    equals the one-rank march bit for bit."""
    N, t, world, steps = 24, 2, 2, 8
    out = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), N, t, steps, out, (64, 4)), nprocs=world, join=True)
    g = CubedSphereGrid(N)
    single = Engine(ShallowWater("tc5"), TileLayout(N, t, 1, ng=2), grid=g, device="cuda", backend="hip", dt=200.0,
                    block=(64, 4))
    single.step(steps)
    L = TileLayout(N, t, world, ng=2)
    for f in range(4):
        glob = assemble_global(L, {r: np.load(os.path.join(out, f"r{r}.npy"))[f] for r in range(world)})
        assert np.array_equal(glob, single.global_field(f)), f


def test_ring_memory_is_pooled_and_zeroed():
    """Uncached ring memory stays with the process: a freed ring is reused by
    the next ring that fits (the allocation zeroes it; handing it back with hipFree was
    followed by corrupted fresh allocations, profiles/r4_ring)."""
    import ctypes
    from stsphere.ops import native
    from stsphere.ops.xgmi import _declare
    L = _declare(native.require_native())
    nb = 3 << 20
    a = ctypes.c_void_p()
    assert L.stsp_xg_alloc(ctypes.c_size_t(nb), ctypes.byref(a)) == 0
    ta = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")   # an ordinary allocation in between
    L.stsp_xg_free(a)
    assert L.stsp_xg_free(a) == -1                 # a second free is refused
    b = ctypes.c_void_p()
    assert L.stsp_xg_alloc(ctypes.c_size_t(nb // 2), ctypes.byref(b)) == 0
    assert b.value == a.value                      # the free ring is reused
    st = (ctypes.c_longlong * 4)()
    L.stsp_xg_pool(st)
    assert st[0] >= 1 and st[2] >= nb
    L.stsp_xg_free(b)
    del ta
