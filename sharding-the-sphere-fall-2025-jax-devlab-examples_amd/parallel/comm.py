"""Halo transports: how remote ghost values reach a rank's ``recv`` buffer.

The reference relies on XLA inserting collectives for the sharded axis
(SURVEY.md 2.3 X1, 2.5).  Here the exchange is explicit point-to-point, one
message per peer per exchange (all fields, all tiles, all halo layers bundled),
in two phases so interior compute can overlap the transfer:

    start(q)  -> pack + post sends/recvs
    finish()  -> wait, return recv [R, F]

Transports
----------
* ``NullTransport``       single rank: everything is a local gather.
* ``TorchDistTransport``  ``torch.distributed`` P2P (gloo on CPU, RCCL on GPU via
                          backend "nccl"); grouped ``batch_isend_irecv``.
* ``VirtualHub``          in-process "virtual devices" (the analogue of the
                          reference's ``--xla_force_host_platform_device_count``,
                          PY:64-68): several ranks in one process stepped in
                          lockstep.
* ``ops.native.NativeRuntime`` owns an RCCL communicator in C++ and runs
  pack -> ncclSend/ncclRecv -> unpack-free gather inside a hipGraph (GPU only).

``staged`` mode (debug) posts the messages stage by stage using
an edge colouring of the device graph, reproducing the reference's "no device
appears twice in the same communication stage" schedule (PDF s.9).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from .layout import RankPlan
from .topology import coloring_to_stages, edge_coloring


def pack_torch(q: torch.Tensor, send_idx: torch.Tensor) -> torch.Tensor:
    """send [Ns, F] = q[:, send_idx].T"""
    return q[:, send_idx].t().contiguous()


class Transport:
    def __init__(self, plan: RankPlan, F: int, dtype, device):
        self.plan = plan
        self.F = F
        self.dtype = dtype
        self.device = device
        self.recv = torch.zeros((max(plan.num_recv, 0), F), dtype=dtype, device=device)
        self.send_idx = torch.as_tensor(plan.send_idx, dtype=torch.long, device=device)
        self.send: Optional[torch.Tensor] = None
        self.pack_fn = pack_torch

    def start(self, q: torch.Tensor) -> None:
        raise NotImplementedError

    def finish(self) -> Optional[torch.Tensor]:
        raise NotImplementedError

    def exchange(self, q: torch.Tensor) -> Optional[torch.Tensor]:
        self.start(q)
        return self.finish()


class NullTransport(Transport):
    def start(self, q):
        pass

    def finish(self):
        return None


class TorchDistTransport(Transport):
    """Grouped P2P over torch.distributed (gloo / RCCL)."""

    def __init__(self, plan, F, dtype, device, group=None, staged: bool = False):
        super().__init__(plan, F, dtype, device)
        self.group = group
        self.staged = staged
        self._reqs = []
        self._stages = None
        if staged:
            self._stages = device_stages(plan)

    def _ops(self, peers=None):
        import torch.distributed as dist
        ops = []
        p = self.plan
        for peer, off, cnt in zip(p.send_peers, p.send_offsets, p.send_counts):
            if peers is None or peer in peers:
                ops.append(dist.P2POp(dist.isend, self.send[off:off + cnt], peer, self.group))
        for peer, off, cnt in zip(p.recv_peers, p.recv_offsets, p.recv_counts):
            if peers is None or peer in peers:
                ops.append(dist.P2POp(dist.irecv, self.recv[off:off + cnt], peer, self.group))
        return ops

    def start(self, q):
        import torch.distributed as dist
        self.send = self.pack_fn(q, self.send_idx)
        if self.staged:
            # stage by stage; each stage completes before the next (debug mode)
            for partners in self._stages:
                ops = self._ops(partners)
                if ops:
                    for r in dist.batch_isend_irecv(ops):
                        r.wait()
            self._reqs = []
            return
        ops = self._ops()
        self._reqs = dist.batch_isend_irecv(ops) if ops else []

    def finish(self):
        for r in self._reqs:
            r.wait()
        self._reqs = []
        return self.recv


def device_stages(plan: RankPlan) -> List[set]:
    """For this rank: the list (per stage) of its partner set, from an edge
    colouring of the whole device graph (identical on every rank)."""
    L = plan.layout
    edges = set()
    for r in range(L.num_ranks):
        pr = L.plan(r)
        for p in pr.peers:
            edges.add((min(r, p), max(r, p)))
    edges = sorted(edges)
    colors = edge_coloring(edges)
    stages = coloring_to_stages(edges, colors)
    out = []
    for st in stages:
        s = set()
        for a, b in st:
            if a == plan.rank:
                s.add(b)
            elif b == plan.rank:
                s.add(a)
        out.append(s)
    return out


class VirtualHub:
    """Shared mailbox for in-process virtual ranks."""

    def __init__(self):
        self.sends: Dict[int, torch.Tensor] = {}
        self.plans: Dict[int, RankPlan] = {}

    def transport(self, plan, F, dtype, device) -> "VirtualTransport":
        self.plans[plan.rank] = plan
        return VirtualTransport(self, plan, F, dtype, device)


class VirtualTransport(Transport):
    def __init__(self, hub: VirtualHub, plan, F, dtype, device):
        super().__init__(plan, F, dtype, device)
        self.hub = hub

    def start(self, q):
        self.hub.sends[self.plan.rank] = self.pack_fn(q, self.send_idx)

    def finish(self):
        p = self.plan
        for peer, off, cnt in zip(p.recv_peers, p.recv_offsets, p.recv_counts):
            pp = self.hub.plans[peer]
            k = pp.send_peers.index(p.rank)
            so, sc = pp.send_offsets[k], pp.send_counts[k]
            assert sc == cnt
            self.recv[off:off + cnt] = self.hub.sends[peer][so:so + sc].to(self.recv.device)
        return self.recv


class NativeBuffers(Transport):
    """Receive buffer for ranks whose halo traffic is driven by the native
    runtime (RCCL inside ``ops.native_runtime.NativeStepper``); Python-side
    stepping is not available through it."""

    def start(self, q):
        raise RuntimeError("halo traffic of this engine is owned by the native runtime; step with NativeStepper")

    def finish(self):
        raise RuntimeError("halo traffic of this engine is owned by the native runtime; step with NativeStepper")


class LoopbackTransport(Transport):
    """Single-rank loopback (layout.loopback): pack and copy into the receive
    buffer in-process (the torch-side twin of an RCCL self send/recv)."""

    def start(self, q):
        self.send = self.pack_fn(q, self.send_idx)

    def finish(self):
        if self.recv.numel():
            self.recv.copy_(self.send)
        return self.recv
