"""Python side of the native step runtime (``ops/csrc/runtime.cpp``).

``NativeStepper(engine)`` turns an engine's integrator period into a C++ op
list (stage kernels; for ranks with remote neighbours also pack + RCCL grouped
send/recv on a high-priority comm stream + interior/boundary split) and hands
stepping to C++: eager, or captured once into a hipGraph and replayed.  The
RCCL communicator is created here (``create_nccl_comm``) and owned natively;
torch.distributed is used only to broadcast the unique id.  The captured graph
plays the role of the reference's second ``jax.jit`` around the composed halo
program (PY:238-246, PDF s.10 "Why two JITs?"): the whole step is recorded
once and replayed without per-op host work.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch

from . import native
from .native import StageDesc

MAX_PEERS = 32
OP_STAGE, OP_PACK, OP_COMM_START, OP_COMM_WAIT, OP_FUSED, OP_IPC_SEND, OP_IPC_WAIT, OP_MARCH3 = 1, 2, 3, 4, 5, 6, 7, 8

_I32x = ctypes.c_int * MAX_PEERS


class StspOp(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int),
        ("phys", ctypes.c_int), ("dtype", ctypes.c_int), ("bx", ctypes.c_int), ("by", ctypes.c_int),
        ("stage", StageDesc),
        ("q", ctypes.c_void_p), ("S", ctypes.c_int), ("F", ctypes.c_int), ("idx", ctypes.c_void_p),
        ("ns", ctypes.c_int), ("send", ctypes.c_void_p),
        ("npeers", ctypes.c_int), ("send_peer", _I32x), ("send_off", _I32x), ("send_cnt", _I32x),
        ("nrecv", ctypes.c_int), ("recv_peer", _I32x), ("recv_off", _I32x), ("recv_cnt", _I32x),
        ("sendbuf", ctypes.c_void_p), ("recvbuf", ctypes.c_void_p), ("slot_elems", ctypes.c_int),
        ("fused", ctypes.c_void_p),
        ("ipc_dst", ctypes.c_void_p * MAX_PEERS), ("ipc_flag", ctypes.c_void_p * MAX_PEERS),
        ("ipc_my_flag", ctypes.c_void_p), ("ipc_counters", ctypes.c_void_p), ("ipc_err", ctypes.c_void_p),
        ("ipc_timeout_ticks", ctypes.c_longlong),
    ]


class StspRtDesc(ctypes.Structure):
    _fields_ = [
        ("nops", ctypes.c_int), ("ops", ctypes.POINTER(StspOp)), ("period", ctypes.c_int),
        ("use_graph", ctypes.c_int), ("graph_periods", ctypes.c_int), ("stream", ctypes.c_void_p),
        ("nccl_comm", ctypes.c_void_p), ("roctx", ctypes.c_int),
    ]


def _declare(L):
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    if L.stsp_desc_size(2) != ctypes.sizeof(StspOp):
        raise RuntimeError(f"StspOp: ctypes mirror is {ctypes.sizeof(StspOp)} bytes, the library's "
                           f"{L.stsp_desc_size(2)} (stale libstsp.so?)")
    L.stsp_rt_create.argtypes = [ctypes.POINTER(StspRtDesc)]
    L.stsp_rt_create.restype = vp
    L.stsp_rt_destroy.argtypes = [vp]
    L.stsp_rt_destroy.restype = None
    L.stsp_rt_run.argtypes = [vp, ci]
    L.stsp_rt_run.restype = ci
    L.stsp_rt_set_dt.argtypes = [vp, cd]
    L.stsp_rt_set_dt.restype = ci
    L.stsp_rt_last_error.argtypes = [vp]
    L.stsp_rt_last_error.restype = ctypes.c_char_p
    L.stsp_nccl_id_bytes.argtypes = []
    L.stsp_nccl_id_bytes.restype = ci
    L.stsp_nccl_unique_id.argtypes = [vp]
    L.stsp_nccl_unique_id.restype = ci
    L.stsp_nccl_comm_init.argtypes = [ci, vp, ci, ci]
    L.stsp_nccl_comm_init.restype = vp
    L.stsp_nccl_comm_destroy.argtypes = [vp]
    L.stsp_nccl_comm_destroy.restype = ci
    L.stsp_nccl_selftest.argtypes = [vp, vp]
    L.stsp_nccl_selftest.restype = ci
    L.stsp_roctx_push.argtypes = [ctypes.c_char_p]
    L.stsp_roctx_push.restype = ci
    L.stsp_roctx_pop.argtypes = []
    L.stsp_roctx_pop.restype = ci
    return L


def lib():
    return _declare(native.require_native())


def create_nccl_comm(rank: int, world: int, device_index: int, group=None) -> int:
    """RCCL communicator owned by the native runtime; the unique id travels
    over the existing torch.distributed process group."""
    import torch.distributed as dist
    L = lib()
    rccl_version()                      # raises (on every rank alike) when RCCL is unusable
    nb = L.stsp_nccl_id_bytes()
    buf = (ctypes.c_char * nb)()
    if rank == 0:
        if L.stsp_nccl_unique_id(buf) != 0:
            raise RuntimeError("ncclGetUniqueId failed")
    dev = torch.device(f"cuda:{device_index}") if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor(list(bytes(buf)), dtype=torch.uint8, device=dev)
    dist.broadcast(t, src=0, group=group)
    raw = bytes(t.cpu().tolist())
    idbuf = (ctypes.c_char * nb).from_buffer_copy(raw)
    comm = L.stsp_nccl_comm_init(world, idbuf, rank, device_index)
    if not comm:
        raise RuntimeError(f"ncclCommInitRank failed: {L.stsp_rccl_error().decode()}")
    return comm


def rccl_version() -> int:
    """Version code (major * 10000 + minor * 100 + patch) of the librccl.so.1
    this process runs (PyTorch's copy when torch is imported first).  Raises
    when it cannot be loaded or lies outside the API range the runtime
    declares (csrc/rccl_abi.h): a header/library mismatch fails loudly here,
    at communicator creation, instead of inside a send."""
    L = lib()
    v = int(L.stsp_rccl_version())
    if v < 0:
        raise RuntimeError(f"RCCL unusable: {L.stsp_rccl_error().decode()}")
    return v


def nccl_selftest(comm: int) -> None:
    L = lib()
    s = torch.cuda.current_stream()
    rc = L.stsp_nccl_selftest(comm, int(s.cuda_stream))
    if rc != 0:
        raise RuntimeError(f"RCCL self send/recv failed ({rc})")


class IpcExchange:
    """IPC copy transport between ranks (``comm: ipc``): the RCCL op list's
    shape (pack -> exchange -> interior blocks -> wait -> boundary blocks)
    with the exchange done by one copy kernel that stores into the peers'
    IPC-mapped receive slots and sets their flags (runtime.cpp
    ``ipc_copy_signal_kernel``; in order on the compute stream, or on the
    comm stream with ``STSP_IPC_FORK=1``), and a spin kernel in place of the
    RCCL wait, so the whole step is graph-captured (RCCL 2.26.6, the copy
    torch loads, crashed under capture: round 3).

    Memory (two allocations per rank, ``xgmi.IpcRing``; peers map both):
    ``nslots`` receive slots of [max num_recv, F] values (read only by the
    boundary blocks, a kernel launched after the wait), and one flag word per
    receive peer (polled inside the wait kernel), both in uncached rings.  Op j of the step's op list fills / reads slot j, so a
    slot is reused ``nslots`` exchanges later: a peer can be at most one
    exchange ahead (its exchange j + 1 starts after its stage j, which waited
    for our exchange j, and our exchange j + 1 is issued after our stage j has
    read slot j), so two slots would do.  Flags and the rank's own counters
    only grow, so replayed graphs and restarts keep their meaning; no priming
    is needed (each stage sends its own input)."""

    def __init__(self, engine, nslots: int, group=None, timeout_s: float = 2.0):
        from .xgmi import IpcRing, _declare
        e = engine
        if nslots < 2:
            raise ValueError("the IPC exchange needs at least two receive slots")
        L = _declare(lib())
        lay = e.layout
        world, rank = lay.num_ranks, e.rank
        self.plans = [lay.plan(p) for p in range(world)]
        plan = self.plans[rank]
        self.F = e.physics.F
        esize = torch.tensor([], dtype=e.dtype).element_size()
        self.esize = esize
        self.nslots = nslots
        rmax = max(max(p.num_recv for p in self.plans), 1)
        self.slot_bytes = -(-rmax * self.F * esize // 256) * 256
        flag_bytes = 256
        peers = sorted(set(int(q) for q in plan.send_peers) | set(int(q) for q in plan.recv_peers) | {rank})
        if len(plan.send_peers) > MAX_PEERS or len(plan.recv_peers) > 64:
            raise RuntimeError("too many peers for the IPC exchange")
        # payload slots and flag words in uncached rings.  A peer on ANOTHER GPU
        # stores into our slot over xGMI, which does not invalidate the lines
        # our L2 kept from reading the same slot nslots exchanges earlier, and
        # the wait kernel's relaxed polls are no acquire: a cached slot could be
        # read stale.  Uncached memory is never held in L2.  Cached
        # slots (STSP_IPC_CACHED=1) were validated only with the ranks sharing
        # one GPU (one L2 hierarchy).
        import os
        cached = os.environ.get("STSP_IPC_CACHED") == "1"
        self.mem = IpcRing(L, e.device, world, rank, peers, nslots * self.slot_bytes, group, cached=cached)
        self.fmem = IpcRing(L, e.device, world, rank, peers, flag_bytes, group)
        self.counters = torch.zeros(4 + MAX_PEERS, dtype=torch.int32, device=e.device)   # runtime.cpp ipc kernels
        self.err = torch.zeros(4, dtype=torch.int32, device=e.device)
        self.timeout_ticks = int(timeout_s * 1e8)
        self.base = self.mem.base
        self.my_flag = self.fmem.base
        # per send peer q: where this rank's cells land in q's slots, and q's flag word for it
        self.dst0, self.flag = [], []
        for q in plan.send_peers:
            qp = self.plans[int(q)]
            idx = list(int(x) for x in qp.recv_peers).index(rank)
            off = int(qp.recv_offsets[idx]) * self.F * esize
            self.dst0.append(int(self.mem.bases[int(q)]) + off)
            self.flag.append(int(self.fmem.bases[int(q)]) + 4 * idx)

    @staticmethod
    def slots_for(engine) -> int:
        """Receive slots of a NativeStepper op list: one per exchange in it."""
        return max(2, engine.integ.period * len(engine.integ.stages))

    def recv_slot(self, j: int) -> int:
        return self.base + (j % self.nslots) * self.slot_bytes

    def check(self) -> None:
        if int(self.err[0].item()) != 0:
            raise RuntimeError("IPC exchange: a peer's cells did not arrive in time (poll timeout)")

    def close(self) -> None:
        for k in ("mem", "fmem"):
            m = getattr(self, k, None)
            if m is not None:
                m.close()
                setattr(self, k, None)


class NativeStepper:
    """Steps an ``Engine(backend='hip')`` entirely from C++.

    Halo traffic between ranks: RCCL (``nccl_comm``; eager, pack + grouped
    send/recv + interior/boundary split) or the direct xGMI exchange
    (``xgmi=XgmiHalo``; one kernel per stage, graph-captured)."""

    def __init__(self, engine, nccl_comm: Optional[int] = None, use_graph: bool = True,
                 steps_per_graph: int = 30, roctx: bool = False, stream: Optional[torch.cuda.Stream] = None,
                 xgmi=None, fused=None, steps_per_launch: int = 1, direct: bool = False, ipc=None, march3=None):
        from .hip_compute import HipCompute
        e = engine
        if not isinstance(e.compute, HipCompute):
            raise RuntimeError("NativeStepper needs an Engine with backend='hip'")
        self.e = e
        self.L = lib()
        hc = e.compute
        plan = e.plan
        self.remote = plan.num_recv > 0 or plan.num_send > 0
        self.xgmi = xgmi
        self.fused = fused
        if fused is not None:
            if xgmi is not None:
                raise RuntimeError("the fused step carries its own exchange")
            self.remote = False      # remote window cells arrive inside the fused kernel
        if xgmi is not None:
            self.remote = False      # the exchange lives inside the stage kernels
        # march3: ops/march3.py::March3Step, the pipelined streaming step of one
        # rank (one march launch + two band launches per step, period 2)
        self.march3 = march3
        if march3 is not None and (fused is not None or xgmi is not None or ipc is not None or self.remote):
            raise RuntimeError("the pipelined march step runs one rank without another step kernel")
        self.ipc = ipc
        if self.remote and not nccl_comm and ipc is None:
            raise RuntimeError("rank has remote neighbours: pass an RCCL communicator (create_nccl_comm) "
                               "or an IpcExchange")
        if len(plan.send_peers) > MAX_PEERS or len(plan.recv_peers) > MAX_PEERS:
            raise RuntimeError("too many peers for the native runtime")
        F = e.physics.F
        self.send = torch.zeros((max(plan.num_send, 1), F), dtype=e.dtype, device=e.device)
        self.send_idx = torch.as_tensor(plan.send_idx, dtype=torch.int32, device=e.device)
        assert (plan.send_idx.size == 0) or int(plan.send_idx.max()) < plan.S
        self.stream = stream or torch.cuda.Stream(device=e.device)
        # fused: ops/fused.py::FusedKernel (temporal blocking), ping-pong between
        # pool[0] and pool[1]: one launch per step, the op list covers two steps;
        # or steps_per_launch (even) steps inside one launch, the op list is that
        # one launch
        self.spl = 1
        if fused is not None and steps_per_launch > 1:
            if steps_per_launch % 2:
                raise ValueError("steps_per_launch must be even")
            self.spl = steps_per_launch
        period = (self.spl if self.spl > 1 else 2) if fused is not None else e.integ.period
        if march3 is not None:
            period = 2
        self.period = period
        ops: List[StspOp] = []
        pool = list(e.pool)
        saved_pool = e.pool
        xj = 0                       # exchanges so far (IPC receive slot of the next one)
        fdescs = [] if fused is None else ([fused.multi_desc(self.spl)] if self.spl > 1 else list(fused.descs))
        for fd in fdescs:
            op = StspOp()
            op.type = OP_FUSED
            op.dtype = fused.dcode
            op.fused = ctypes.addressof(fd)
            ops.append(op)
        if march3 is not None:
            ops.extend(march3.ops())
        for _ in range(period if (fused is None and march3 is None) else 0):
            e.pool = pool
            for st in e.integ.stages:
                if xgmi is not None:
                    ops.append(self._stage_op(xgmi.fill(hc.desc(st, e.dt, None, hc.nblocks))))
                    continue
                if not hc.remote:
                    ops.append(self._stage_op(hc.desc(st, e.dt, None, hc.nblocks)))
                    continue
                op = StspOp()
                op.type = OP_PACK
                op.dtype = hc.dcode
                op.q = native.ptr(pool[st.Q])
                op.S = plan.S
                op.F = F
                op.idx = native.ptr(self.send_idx)
                op.ns = plan.num_send
                op.send = native.ptr(self.send)
                ops.append(op)
                if ipc is not None:
                    ops.append(self._ipc_send_op(hc.dcode, F, xj))
                else:
                    ops.append(self._comm_op(hc.dcode, F))
                if hc.blk_interior.numel():
                    ops.append(self._stage_op(hc.desc(st, e.dt, hc.blk_interior, hc.blk_interior.numel())))
                w = StspOp()
                if ipc is not None:
                    w.type = OP_IPC_WAIT
                    w.nrecv = len(plan.recv_peers)
                    w.ipc_my_flag = ipc.my_flag
                    w.ipc_counters = native.ptr(ipc.counters)
                    w.ipc_err = native.ptr(ipc.err)
                    w.ipc_timeout_ticks = ipc.timeout_ticks
                else:
                    w.type = OP_COMM_WAIT
                ops.append(w)
                if hc.blk_boundary.numel():
                    bd = hc.desc(st, e.dt, hc.blk_boundary, hc.blk_boundary.numel(), remote=True)
                    if ipc is not None:
                        bd.recv = ipc.recv_slot(xj)       # this exchange's receive slot
                    ops.append(self._stage_op(bd))
                xj += 1
            pool = [pool[r] for r in e.integ.rotation]
        e.pool = saved_pool
        self._ops = (StspOp * len(ops))(*ops)
        d = StspRtDesc()
        d.nops = len(ops)
        d.ops = self._ops
        d.period = period
        # hipGraph capture of the RCCL P2P ops segfaults inside the RCCL 2.26.6 that
        # ships with this PyTorch (measured: eager loopback exact, captured crash), so
        # op lists with comm run eagerly from C++ unless STSP_GRAPH_COMM=1.
        import os
        graph_ok = (not self.remote) or ipc is not None or os.environ.get("STSP_GRAPH_COMM") == "1"
        self.use_graph = bool(use_graph and graph_ok)
        # Graph container: the C++ runtime's eager op list recorded by
        # torch.cuda.graph and replayed on torch's current stream.  Measured on
        # MI355X (tools/runtime_ab.py, C96): 17.2 us/step, against 20-21 us/step
        # for the same launches replayed on a side stream (C++-side graph or
        # torch graph alike; capture mode, instantiate flags and upload made no
        # difference).  STSP_NATIVE_GRAPH=1 selects the C++-side graph.
        self._cxx_graph = self.use_graph and os.environ.get("STSP_NATIVE_GRAPH") == "1"
        d.use_graph = 1 if self._cxx_graph else 0
        self.graph_periods = max(1, steps_per_graph // period)
        d.graph_periods = self.graph_periods
        self._graphs = {}          # (periods, copy) -> torch.cuda.CUDAGraph
        self._primed = set()       # (periods, copy) replayed at least once
        self._next_copy = {}       # periods -> copy the next replay of that length uses
        self._pool0 = list(e.pool)  # construction order = the op list's buffer pointers
        self.stats = {"graph_steps": 0, "eager_steps": 0, "replays": 0, "direct_steps": 0, "launches": 0}
        # direct (fused runtime only): every period is ONE kernel launch issued
        # from Python through ctypes on torch's current stream, no graph.  A
        # fused multi-step period is a single kernel, so a graph around it buys
        # nothing; measured at C96 20/5 (tools/launch_probe.py,
        # profiles/r3_march/launch_probe.json): 13.70 us/step direct against
        # 14.22 replaying the one-node graph (hipGraphLaunch's host floor)
        if direct and fused is None:
            raise ValueError("direct launches are the fused runtime's")
        self.direct = bool(direct)
        self._dev_index = e.device.index if e.device.index is not None else (
            torch.cuda.current_device() if e.device.type == "cuda" else 0)
        if self.direct:
            self.use_graph = False
        self._warmed = False
        d.stream = int(self.stream.cuda_stream)
        d.nccl_comm = nccl_comm or 0
        d.roctx = 1 if roctx else 0
        self._desc = d
        self.h = self.L.stsp_rt_create(ctypes.byref(d))
        if not self.h:
            raise RuntimeError("stsp_rt_create failed")

    def _stage_op(self, sd: StageDesc) -> StspOp:
        hc = self.e.compute
        op = StspOp()
        op.type = OP_STAGE
        op.phys, op.dtype, op.bx, op.by = hc.phys_id, hc.dcode, hc.bx, hc.by
        op.stage = sd
        return op

    def _ipc_send_op(self, dcode: int, F: int, j: int) -> StspOp:
        p = self.e.plan
        ipc = self.ipc
        op = StspOp()
        op.type = OP_IPC_SEND
        op.dtype = dcode
        op.npeers = len(p.send_peers)
        for k, (off, cnt) in enumerate(zip(p.send_offsets, p.send_counts)):
            op.send_off[k], op.send_cnt[k] = off, cnt
            op.ipc_dst[k] = ipc.dst0[k] + (j % ipc.nslots) * ipc.slot_bytes
            op.ipc_flag[k] = ipc.flag[k]
        op.sendbuf = native.ptr(self.send)
        op.slot_elems = F
        op.ipc_counters = native.ptr(ipc.counters)
        return op

    def _comm_op(self, dcode: int, F: int) -> StspOp:
        p = self.e.plan
        op = StspOp()
        op.type = OP_COMM_START
        op.dtype = dcode
        op.npeers = len(p.send_peers)
        for k, (peer, off, cnt) in enumerate(zip(p.send_peers, p.send_offsets, p.send_counts)):
            op.send_peer[k], op.send_off[k], op.send_cnt[k] = peer, off, cnt
        op.nrecv = len(p.recv_peers)
        for k, (peer, off, cnt) in enumerate(zip(p.recv_peers, p.recv_offsets, p.recv_counts)):
            op.recv_peer[k], op.recv_off[k], op.recv_cnt[k] = peer, off, cnt
        op.sendbuf = native.ptr(self.send)
        op.recvbuf = native.ptr(self.e.transport.recv)
        op.slot_elems = F
        return op

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self.L.stsp_rt_last_error(self.h)
            raise RuntimeError(f"native runtime {what} failed ({rc}): {msg.decode() if msg else ''}")

    def check(self) -> None:
        if self.xgmi is not None:
            self.xgmi.check()
        if self.ipc is not None:
            self.ipc.check()
        if self.fused is not None:
            self.fused.check()

    def err_words(self) -> List[torch.Tensor]:
        """Device error words the kernels set on a timed-out wait (non-zero:
        the state is not to be trusted); ``check()`` raises on them."""
        out = []
        if self.xgmi is not None:
            out.append(self.xgmi.err)
        if self.ipc is not None:
            out.append(self.ipc.err)
        if self.fused is not None:
            out.append(self.fused.tens["err"])
        return out

    def _run_native(self, nsteps: int) -> None:
        """Eager op list on self.stream, ordered after and before torch's
        current stream."""
        if nsteps:
            cur = torch.cuda.current_stream(self.e.device)
            self.stream.wait_stream(cur)
            self._check(self.L.stsp_rt_run(self.h, nsteps), "run")
            cur.wait_stream(self.stream)
            self.stats["eager_steps"] += nsteps

    def _warm(self) -> None:
        """Lazy one-time setup (RCCL, streams, code objects) must not happen
        under capture: run one period eagerly on a scratch copy of the state
        (the state, time and step count are left unchanged)."""
        if self._warmed:
            return
        saved = self._save()
        self._run_native(self.period)
        self.stats["eager_steps"] -= self.period     # not a step of the run
        torch.cuda.synchronize(self.e.device)
        self._restore(saved)
        self._warmed = True

    def _save(self):
        return [b.clone() for b in self._pool0]

    def _restore(self, saved) -> None:
        for b, s in zip(self._pool0, saved):
            b.copy_(s)
        torch.cuda.synchronize(self.e.device)
        if self.xgmi is not None:
            self.xgmi.prime()          # re-deliver the remote ghosts of the restored state (collective)
        if self.fused is not None:
            self.fused.prime()         # the same for the fused step's remote window cells

    def _graph(self, periods: int, copy: int = 0):
        """hipGraph of exactly ``periods`` integrator periods (recorded once,
        cached by length; recorded launches carry the current dt).  Two
        copies per length: a graph exec launched again while its previous
        launch is still running holds the host until that launch is done, so
        back-to-back chunks of one length alternate between the copies and
        the host stays a chunk ahead of the GPU (profiles/r2_ensemble)."""
        key = (periods, copy)
        g = self._graphs.get(key)
        if g is None:
            self._warm()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream):
                self._check(self.L.stsp_rt_run(self.h, periods * self.period), "capture")   # recorded, not executed
            self._graphs[key] = g
            self._primed.discard(key)
        return g

    def plan(self, nsteps: int) -> List[int]:
        """Graph lengths (in periods) that ``run(nsteps)`` replays: full
        ``steps_per_graph`` chunks, then one graph for the remainder, so every
        step of a run is a graph replay whatever ``nsteps`` is."""
        periods = nsteps // self.period
        k = self.graph_periods
        chunks = [k] * (periods // k)
        if periods % k:
            chunks.append(periods % k)
        return chunks

    def _dev_stream(self) -> int:
        return native.current_stream_handle(self._dev_index)

    def _run_direct(self, nsteps: int) -> None:
        """nsteps (a multiple of the period) as direct fused launches."""
        st = self._dev_stream()
        for _ in range(nsteps // self.period):
            if self.spl > 1:
                self.fused.launch(0, st, nsteps=self.spl)
                self.stats["launches"] += 1
            else:
                self.fused.launch(0, st)
                self.fused.launch(1, st)
                self.stats["launches"] += 2
        self.stats["direct_steps"] += nsteps

    def prepare(self, nsteps: int, prime: bool = True) -> None:
        """Record every graph ``run(nsteps)`` will replay and (prime=True)
        replay each once on a scratch copy of the state, so the first timed
        replay pays neither capture, instantiation nor upload.  The state,
        time and step count are unchanged.  With the direct xGMI exchange this
        is collective (the restore re-primes the rings)."""
        if self.direct:
            # one untimed pass of the same launches on a scratch copy (first-use
            # costs), the remainder launch of a chunk that is not a whole number
            # of periods included (its descriptor is built here, not in the run)
            rem = nsteps % self.period
            if rem >= 2 and self.spl > 1:
                self.fused.multi_desc(rem - rem % 2)
            if prime and nsteps:
                saved = self._save()
                if nsteps // self.period:
                    self._run_direct((nsteps // self.period) * self.period)
                if rem >= 2 and self.spl > 1:
                    self.fused.launch(0, int(torch.cuda.current_stream(self.e.device).cuda_stream),
                                      nsteps=rem - rem % 2)
                torch.cuda.synchronize(self.e.device)
                self._restore(saved)
                self.stats["direct_steps"] = 0
                self.stats["launches"] = 0
            return
        if not self.use_graph or self._cxx_graph:
            return
        todo = []
        for c in self.plan(nsteps):
            for copy in (0, 1):
                key = (c, copy)
                self._graph(c, copy)
                if key not in self._primed and key not in todo:
                    todo.append(key)
        if prime and todo:
            saved = self._save()
            for key in todo:
                self._graphs[key].replay()
                self._primed.add(key)
            torch.cuda.synchronize(self.e.device)
            self._restore(saved)

    def _run(self, nsteps: int) -> None:
        """nsteps (a multiple of the period)."""
        if self.direct:
            self._run_direct(nsteps)
            return
        if not self.use_graph or self._cxx_graph:
            self._run_native(nsteps)
            return
        # replay on torch's current stream: measured 17.2 us/step at C96 there
        # against 20-21 us/step when the same graph is launched on a side stream
        for c in self.plan(nsteps):
            copy = self._next_copy.get(c, 0)
            self._graph(c, copy).replay()
            self._primed.add((c, copy))
            self._next_copy[c] = 1 - copy
            self.stats["graph_steps"] += c * self.period
            self.stats["replays"] += 1

    def _sync_pool(self) -> None:
        """The op list holds the buffer pointers of the construction-order
        pool.  Engine.step rotates ``e.pool`` (period > 1 integrators), so after
        a partial period copy the rotated buffers back into construction order
        (a rotated pool made the next native run read stale state)."""
        e = self.e
        if all(a is b for a, b in zip(e.pool, self._pool0)):
            return
        vals = [b.clone() for b in e.pool]
        for b, v in zip(self._pool0, vals):
            b.copy_(v)
        e.pool = list(self._pool0)

    def run(self, nsteps: int) -> None:
        e = self.e
        self._sync_pool()
        full = (nsteps // self.period) * self.period
        if full:
            self._run(full)
            e.time += full * e.dt
            e.step_count += full
        if nsteps - full:
            if self.fused is not None:
                # remainder: an odd first step copied back to pool[0], then the even
                # part in one launch (the multi-step kernel runs last, as in the
                # next full period)
                cur = torch.cuda.current_stream(e.device)
                rem = nsteps - full
                if rem % 2:
                    self.fused.launch(0, int(cur.cuda_stream))
                    e.pool[0].copy_(e.pool[1])
                if rem >= 2 and self.spl > 1:
                    self.fused.launch(0, int(cur.cuda_stream), nsteps=rem - rem % 2)
                elif rem >= 2:
                    for _ in range(rem // 2):
                        self.fused.launch(0, int(cur.cuda_stream))
                        self.fused.launch(1, int(cur.cuda_stream))
                e.time += rem * e.dt
                e.step_count += rem
            else:
                e.step(nsteps - full)
            self.stats["eager_steps"] += nsteps - full
            self._sync_pool()

    def set_dt(self, dt: float) -> None:
        self.e.dt = dt
        if self.fused is not None:
            self.fused.set_dt(dt)
        self._check(self.L.stsp_rt_set_dt(self.h, dt), "set_dt")
        self._graphs = {}     # recorded launches carry the old dt
        self._primed = set()
        self._next_copy = {}

    def close(self) -> None:
        self._graphs = {}
        if getattr(self, "h", None):
            self.L.stsp_rt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
