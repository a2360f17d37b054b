"""Native C++ step runtime (hipGraph + RCCL) on one GPU.

The loopback layout routes every ghost through pack -> RCCL grouped
send/recv (to self) -> receive-buffer gather, i.e. the complete multi-GPU
path, on a single MI355X."""
import os
import socket

import pytest
import torch

from stsphere.engine import Engine
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.models.advection import Advection
from stsphere.parallel.comm import NativeBuffers
from stsphere.parallel.layout import TileLayout

pytestmark = pytest.mark.gpu


def _single(N=24, t=2, phys=lambda: ShallowWater("tc5"), integ="ssprk3"):
    g = CubedSphereGrid(N)
    return g, Engine(phys(), TileLayout(N, t, 1, ng=2), grid=g, device="cuda", backend="hip", integrator=integ)


@pytest.mark.parametrize("use_graph", [True, False])
@pytest.mark.parametrize("integ", ["ssprk3", "rk4", "euler"])
def test_native_stepper_matches_engine(use_graph, integ):
    from stsphere.ops.native_runtime import NativeStepper
    g, a = _single(integ=integ)
    _, b = _single(integ=integ)
    ns = NativeStepper(b, use_graph=use_graph, steps_per_graph=4)
    a.step(10)
    ns.run(10)
    torch.cuda.synchronize()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert b.step_count == 10
    ns.close()


@pytest.mark.parametrize("integ", ["euler", "ssprk3"])
def test_odd_chunks_keep_runner_and_pool_in_sync(integ):
    """run(3); run(3) == Engine.step(6) even when a chunk is not a multiple of
    the integrator period (euler ping-pongs its buffers: ADVICE r1)."""
    from stsphere.engine import GraphStepper
    from stsphere.ops.native_runtime import NativeStepper
    _, a = _single(integ=integ)
    _, b = _single(integ=integ)
    _, c = _single(integ=integ)
    ns = NativeStepper(b, use_graph=True, steps_per_graph=4)
    gs = GraphStepper(c, steps_per_graph=2)
    a.step(6)
    for _ in range(2):
        ns.run(3)
        gs.run(3)
    torch.cuda.synchronize()
    assert torch.equal(a.tiles_view(), b.tiles_view())
    assert torch.equal(a.tiles_view(), c.tiles_view())
    assert b.step_count == 6 and c.step_count == 6
    ns.close()


def test_short_run_replays_a_graph():
    """run(20) with the default 30-step graph length replays recorded graphs
    only (r1: 20 // 30 = 0 graphs, so every step ran eagerly)."""
    from stsphere.ops.native_runtime import NativeStepper
    _, a = _single()
    _, b = _single()
    ns = NativeStepper(b, use_graph=True, steps_per_graph=30)
    ns.prepare(20)
    assert b.step_count == 0 and torch.equal(a.tiles_view(), b.tiles_view())   # prepare leaves the state alone
    s0 = dict(ns.stats)
    ns.run(20)
    a.step(20)
    torch.cuda.synchronize()
    assert ns.stats["eager_steps"] == s0["eager_steps"]
    assert ns.stats["graph_steps"] - s0["graph_steps"] == 20 and ns.stats["replays"] - s0["replays"] == 1
    assert torch.equal(a.tiles_view(), b.tiles_view())
    ns.run(35)      # one 30-step graph + a 5-step graph
    a.step(35)
    torch.cuda.synchronize()
    assert ns.stats["eager_steps"] == s0["eager_steps"]
    assert torch.equal(a.tiles_view(), b.tiles_view())
    ns.close()


@pytest.fixture(scope="module")
def nccl_comm():
    import torch.distributed as dist
    from stsphere.ops import native_runtime as nr
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    comm = nr.create_nccl_comm(0, 1, 0)
    yield comm
    nr.lib().stsp_nccl_comm_destroy(comm)
    dist.destroy_process_group()


def test_rccl_selftest(nccl_comm):
    from stsphere.ops.native_runtime import nccl_selftest
    nccl_selftest(nccl_comm)


@pytest.mark.parametrize("use_graph", [False, True])
@pytest.mark.parametrize("phys", ["swe", "adv"])
def test_rccl_loopback_full_multigpu_path(nccl_comm, use_graph, phys):
    from stsphere.ops.native_runtime import NativeStepper
    mk = {"swe": lambda: ShallowWater("tc5"), "adv": lambda: Advection()}[phys]
    g, ref = _single(phys=mk)
    L = TileLayout(24, 2, 1, ng=2, loopback=True)
    p = L.plan(0)
    F = ref.physics.F
    e = Engine(mk(), L, grid=g, device="cuda", backend="hip", dt=ref.dt,
               transport=NativeBuffers(p, F, torch.float64, torch.device("cuda")))
    assert e.compute.remote and e.compute.blk_boundary.numel() > 0
    ns = NativeStepper(e, nccl_comm=nccl_comm, use_graph=use_graph, steps_per_graph=3)
    assert not ns.use_graph      # comm op lists run eagerly (RCCL capture crash, see native_runtime.py)
    ref.step(6)
    ns.run(6)
    torch.cuda.synchronize()
    assert torch.equal(ref.tiles_view(), e.tiles_view())
    ns.close()



@pytest.mark.parametrize("use_graph", [True, False])
@pytest.mark.parametrize("integ", ["ssprk3", "rk4"])
def test_ipc_copy_loopback_full_multigpu_path(use_graph, integ):
    """The IPC copy transport (pack -> one copy kernel into the peer's receive
    slot, which also stores the peer's flag -> interior blocks -> spin-wait
    kernel -> boundary blocks) on the loopback layout, where every ghost
    crosses it: bitwise equal to the single-rank engine, and, unlike the RCCL
    op list, recorded into a graph and replayed."""
    from stsphere.ops.native_runtime import IpcExchange, NativeStepper
    g, ref = _single(integ=integ)
    L = TileLayout(24, 2, 1, ng=2, loopback=True)
    p = L.plan(0)
    e = Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip", dt=ref.dt, integrator=integ,
               transport=NativeBuffers(p, 4, torch.float64, torch.device("cuda")))
    assert e.compute.remote and e.compute.blk_boundary.numel() > 0
    ipc = IpcExchange(e, IpcExchange.slots_for(e))
    ns = NativeStepper(e, use_graph=use_graph, steps_per_graph=3, ipc=ipc)
    assert ns.use_graph == use_graph
    ref.step(9)
    ns.run(9)
    torch.cuda.synchronize()
    ns.check()
    assert torch.equal(ref.tiles_view(), e.tiles_view())
    if use_graph:
        assert ns.stats["graph_steps"] >= 6 and ns.stats["eager_steps"] <= 3
    ns.close()
    ipc.close()


@pytest.mark.parametrize("phys,dtype", [("adv", torch.float32), ("adv", torch.float64), ("swe", torch.float32)])
def test_ipc_copy_kernel_word_sizes(phys, dtype):
    """The IPC copy kernel (runtime.cpp::ipc_copy_signal_kernel) copies
    16-byte words when every payload allows, else 4-byte words: one field in
    fp32 (tracer advection) gives payloads that are not 16-byte multiples.
    Each case is bitwise equal to the single-rank engine of the same dtype,
    graph-replayed."""
    from stsphere.ops.native_runtime import IpcExchange, NativeStepper
    mk = {"swe": lambda: ShallowWater("tc5"), "adv": lambda: Advection()}[phys]
    g = CubedSphereGrid(24)
    ref = Engine(mk(), TileLayout(24, 2, 1, ng=2), grid=g, dtype=dtype, device="cuda", backend="hip")
    L = TileLayout(24, 2, 1, ng=2, loopback=True)
    F = ref.physics.F
    e = Engine(mk(), L, grid=g, dtype=dtype, device="cuda", backend="hip", dt=ref.dt,
               transport=NativeBuffers(L.plan(0), F, dtype, torch.device("cuda")))
    ipc = IpcExchange(e, IpcExchange.slots_for(e))
    ns = NativeStepper(e, use_graph=True, steps_per_graph=3, ipc=ipc)
    ref.step(6)
    ns.run(6)
    torch.cuda.synchronize()
    ns.check()
    assert torch.equal(ref.tiles_view(), e.tiles_view())
    ns.close()
    ipc.close()
