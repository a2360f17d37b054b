"""Direct xGMI halo exchange: stage kernels store remote ghost cells straight
into the neighbour GPU's memory, with no RCCL and no host in the loop.

Why (BASELINE configs "C96 on 6 MI355X", "C180 on 8"):
at C96 a stage takes about 6.5 us on one GPU.  An RCCL grouped send/recv per
stage costs as much as a whole stage.  It is host-driven, and RCCL 2.26 in
this image cannot be captured into a hipGraph (ops/native_runtime.py).
MI355X GPUs in a node are fully connected by xGMI, and a GPU can store
directly into a peer's HBM through a dmabuf IPC mapping.  The exchange
therefore becomes part of the stage kernel itself (ops/csrc/stage_kernel.hip,
XG variant).  It is the explicit form of the cross-device transfer the
reference leaves to XLA when ``exchange_edge_pair`` (PY:166-197) reads one
sharded face and writes another:

* Every rank owns one uncached allocation holding ``[world]`` u64 arrival
  counters and a 4-slot receive ring (``ring_slots x F`` values per slot).
  Peers map it with ``hipIpcOpenMemHandle``.
* A block whose cells are ghosts of another rank stores them into that rank's
  ring slot ``(epoch + 1) % 4``.  The push map carries the destination:
  ``-2 - (peer << 24 | slot)``.
* Hand-off (``stsp_xg_protocol()``, compile-time):

  - tagged granules (1): every 32-bit word of a ghost travels as one 8-byte
    ``{tag = epoch + 1, payload}`` atomic store; the consumer thread re-reads
    its granules until every tag matches.  The data is the flag: no drain, no
    counter, no separate poll round trip.
  - arrival counters (0): the producer's waves drain their stores, then one
    lane per peer adds 1 to that peer's counter (system-scope release).  A
    block that reads remote ghosts polls the counters of those peers until
    ``counter[p] >= epoch * nprod[p]``.  ``nprod[p]`` is the number of producer
    blocks on p that feed this rank.

  Either wait is bounded by a timeout that sets ``err``; after that every wait
  falls through.
* ``epoch`` is a per-block count of completed stages.  Tags and counters never
  reset.

Four slots make the ring race-free: a peer can have started at most two stages
past a rank's current stage (the proof is at STSP_XG_SLOTS in the kernel), so
it never writes the slot that rank still reads.  The whole step is plain
kernels, so multi-GPU steps are captured in a hipGraph like single-GPU ones.

``XgmiPlan`` is the host-side index math (numpy only, tested on CPU).
``XgmiHalo`` owns the memory, the IPC mappings and the initial delivery.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch

from ..parallel.layout import TileLayout, corner_own_index, corner_xy

CNT_BYTES = 256          # counter block at the start of each rank's allocation (<= 32 ranks)
MAX_WORLD = 32
SLOT_BITS = 24


def _side_cell(s2: np.ndarray, kk: np.ndarray, pp: np.ndarray, n: int):
    """(side, layer, pos) of a push entry -> own-cell (i, j); inverse of the
    kernel's push lookup (stage_kernel.hip, phase 0)."""
    i = np.select([s2 == 0, s2 == 1, s2 == 2], [kk, n - 1 - kk, pp], pp)
    j = np.select([s2 == 0, s2 == 1, s2 == 2], [pp, pp, kk], n - 1 - kk)
    return i, j


class XgmiPlan:
    """Index tables of the direct exchange for one rank (host side)."""

    def __init__(self, layout: TileLayout, rank: int, bx: int, by: int, halo: int):
        L = layout
        self.layout, self.rank, self.bx, self.by, self.halo = L, rank, bx, by, halo
        world = L.num_ranks
        if world > MAX_WORLD:
            raise ValueError(f"direct xGMI halo supports at most {MAX_WORLD} ranks")
        plan = L.plan(rank)
        self.plan = plan
        n, g = plan.n, plan.ng
        self.nbx, self.nby = -(-n // bx), -(-n // by)
        self.nblocks = plan.T * self.nbx * self.nby
        tnbr = L.tile_neighbors()
        plans = [L.plan(p) for p in range(world)]
        self.ring_slots = max(1, max(p.num_recv for p in plans))
        if self.ring_slots >= (1 << SLOT_BITS):
            raise ValueError("receive ring too large for the push-map encoding")

        # ---- producer side: my cells that are remote ghosts of rank p ----------
        push = plan.push_map.astype(np.int64).copy()
        src_l, code_l, feed_blk, feed_peer = [], [], [], []
        for p in plan.send_peers:
            pp_ = plans[p]
            gs = L.ghost_sources(p)                          # [Tp,4,g,n] global source cells
            tid, _, _ = L.locate(gs)
            sel = (np.asarray(L.owner)[tid] == rank) & (pp_.ghost_map < 0)
            if not sel.any():
                continue
            slot = (-1 - pp_.ghost_map[sel]).astype(np.int64)
            c = gs[sel]
            tid2, i2, j2 = L.locate(c)
            recv_tile = np.asarray(pp_.tiles)[np.nonzero(sel)[0]]
            # side of the source tile facing the receiving tile with the cell inside the strip
            cand = np.stack([(i2, j2), (n - 1 - i2, j2), (j2, i2), (n - 1 - j2, i2)], 0)   # [4, 2, M]
            kk_all, pp_all = cand[:, 0], cand[:, 1]
            ok = (tnbr[tid2].T == recv_tile[None, :]) & (kk_all < g)
            if not ok.any(axis=0).all():
                raise AssertionError("a remote ghost slot has no feeding strip cell")
            s2 = np.argmax(ok, axis=0)
            m = np.arange(len(c))
            kk, pp = kk_all[s2, m], pp_all[s2, m]
            li = L._local_arr[tid2]
            code = (np.int64(p) << SLOT_BITS) | slot
            cur = push[li, s2, kk, pp]
            if not ((cur == -1) | (cur == -2 - code)).all():
                raise AssertionError("push-map collision between a local and a remote ghost")
            push[li, s2, kk, pp] = -2 - code
            src_l.append(L.local_flat(c))
            code_l.append(code)
            ii, jj = _side_cell(s2, kk, pp, n)
            feed_blk.append((li * self.nby + jj // by) * self.nbx + ii // bx)
            feed_peer.append(np.full(len(c), p, dtype=np.int64))
        self.push = push.astype(np.int32)
        # carried corner ghosts of peers (parallel/layout.py::corner_sources):
        # their own push table, with the same remote codes
        cpush = plan.corner_push.astype(np.int64).copy()
        for p in plan.send_peers:
            pp_ = plans[p]
            cs = L.corner_sources(p)
            sel = pp_.corner_carried & (pp_.corner_map < 0)
            if not sel.any():
                continue
            c = cs[sel]
            mine = np.asarray(L.owner)[L.locate(c)[0]] == rank
            if not mine.any():
                continue
            c = c[mine]
            slot = (-1 - pp_.corner_map[sel][mine]).astype(np.int64)
            tid2, i2, j2 = L.locate(c)
            qo, ao, bo = corner_own_index(i2, j2, n, g)
            li = L._local_arr[tid2]
            code = (np.int64(p) << SLOT_BITS) | slot
            cur = cpush[li, qo, ao, bo]
            if not ((cur == -1) | (cur == -2 - code)).all():
                raise AssertionError("corner push collision")
            cpush[li, qo, ao, bo] = -2 - code
            src_l.append(L.local_flat(c))
            code_l.append(code)
            feed_blk.append((li * self.nby + j2 // by) * self.nbx + i2 // bx)
            feed_peer.append(np.full(len(c), p, dtype=np.int64))
        self.cpush = cpush.astype(np.int32)
        if src_l:
            src = np.concatenate(src_l)
            code = np.concatenate(code_l)
            # one prime entry per (source cell, destination slot)
            key = np.unique(np.stack([src, code], 1), axis=0)
            self.prime_src = key[:, 0].astype(np.int32)
            self.prime_code = key[:, 1].astype(np.int32)
            fb, fp = np.concatenate(feed_blk), np.concatenate(feed_peer)
        else:
            self.prime_src = np.zeros(0, np.int32)
            self.prime_code = np.zeros(0, np.int32)
            fb = fp = np.zeros(0, np.int64)
        bmask = np.zeros((self.nblocks, 2), dtype=np.int64)
        np.bitwise_or.at(bmask[:, 1], fb, np.left_shift(1, fp))

        # ---- consumer side ----------------------------------------------------
        gm = plan.ghost_map
        slot_peer = np.full(max(plan.num_recv, 1), -1, dtype=np.int64)
        for p, off, cnt in zip(plan.recv_peers, plan.recv_offsets, plan.recv_counts):
            slot_peer[off:off + cnt] = p
        NG = halo
        rcorner = plan.remote_corners()
        cxy = []
        for t in range(plan.T):
            qq, aa, bb = np.nonzero(rcorner[t])
            cxy.append(corner_xy(qq, aa, bb, n))
        for t in range(plan.T):
            for yb in range(self.nby):
                y0 = yb * by
                for xb in range(self.nbx):
                    x0 = xb * bx
                    bits = 0
                    rows = slice(max(0, y0 - NG), min(n, y0 + by + NG))
                    cols = slice(max(0, x0 - NG), min(n, x0 + bx + NG))
                    parts = []
                    if x0 < NG:
                        parts.append(gm[t, 0, :NG - x0, rows])
                    if x0 + bx + NG > n:
                        parts.append(gm[t, 1, :min(NG, x0 + bx + NG - n), rows])
                    if y0 < NG:
                        parts.append(gm[t, 2, :NG - y0, cols])
                    if y0 + by + NG > n:
                        parts.append(gm[t, 3, :min(NG, y0 + by + NG - n), cols])
                    cm = plan.corner_map[t][rcorner[t]]
                    cx, cy = cxy[t]
                    inw = (cx >= x0 - NG) & (cx < x0 + bx + NG) & (cy >= y0 - NG) & (cy < y0 + by + NG)
                    parts.append(cm[inw])
                    for q in parts:
                        r = q[q < 0]
                        for p in np.unique(slot_peer[-1 - r]):
                            bits |= 1 << int(p)
                    bmask[(t * self.nby + yb) * self.nbx + xb, 0] = bits
        self.bmask = bmask.astype(np.int32)

        # producer blocks of each peer that feed this rank (cells of my ghosts, all layers)
        self.nprod = np.zeros(MAX_WORLD, dtype=np.int64)
        gs = L.ghost_sources(rank)
        cs = L.corner_sources(rank)
        for p in plan.recv_peers:
            sel = gm < 0
            c = np.concatenate([gs[sel], cs[rcorner]])
            tid, i, j = L.locate(c)
            own = np.asarray(L.owner)[tid]
            c_t, c_i, c_j = tid[own == p], i[own == p], j[own == p]
            blk = (L._local_arr[c_t] * self.nby + c_j // by) * self.nbx + c_i // bx
            self.nprod[p] = len(np.unique(blk))


def refuse_if_forced() -> None:
    """Test hook of the transport fallback chain (xgmi -> ipc -> rccl):
    ``STSP_FAIL_XGMI=1`` makes every direct-ring setup raise on every rank
    alike, as a node without peer IPC would."""
    import os
    if os.environ.get("STSP_FAIL_XGMI") == "1":
        raise RuntimeError("direct xGMI ring setup refused (STSP_FAIL_XGMI=1 test hook)")


class XgmiHalo:
    """Memory, IPC mappings and initial delivery of the direct exchange for
    one ``Engine(backend='hip')``; ``fill(desc)`` turns a stage descriptor into
    its XG form."""

    def __init__(self, engine, group=None, timeout_s: float = 2.0):
        from . import native
        refuse_if_forced()
        from .hip_compute import HipCompute
        e = engine
        if not isinstance(e.compute, HipCompute):
            raise RuntimeError("XgmiHalo needs an Engine with backend='hip'")
        self.e = e
        self.group = group
        hc = e.compute
        L = self._lib = _declare(native.require_native())
        world = e.layout.num_ranks
        self.world = world
        self.rank = e.rank
        hc.use_march_with_xgmi()         # large ranks stream (march_kernel.hip reads the ring itself)
        self.xp = XgmiPlan(e.layout, e.rank, hc.bx, hc.by, e.physics.halo)
        self._check_chain(e.integ)
        dev = e.device
        F = e.physics.F
        self.esize = torch.tensor([], dtype=e.dtype).element_size()
        self.protocol = int(L.stsp_xg_protocol())
        self.slots = int(L.stsp_xg_slots())
        if self.protocol == 1:   # 8-byte granules, one per 32-bit word
            self.ring = self.xp.ring_slots * F * (self.esize // 4)
            nbytes = CNT_BYTES + self.slots * self.ring * 8
        else:
            self.ring = self.xp.ring_slots * F
            nbytes = CNT_BYTES + self.slots * self.ring * self.esize
        self.base = None
        peers = sorted(set(self.xp.plan.send_peers) | set(self.xp.plan.recv_peers))
        self.mem = IpcRing(L, dev, world, self.rank, peers, nbytes, group)
        self.base = self.mem.base
        bases = self.mem.bases
        distributed = self.mem.distributed
        pr = np.zeros(MAX_WORLD, dtype=np.int64)
        pc = np.zeros(MAX_WORLD, dtype=np.int64)
        for p, b in bases.items():
            pr[p] = b + CNT_BYTES
            pc[p] = b + 8 * self.rank
        self.peer_ring = torch.as_tensor(pr, device=dev)
        self.peer_cnt = torch.as_tensor(pc, device=dev)
        self.nprod = torch.as_tensor(self.xp.nprod, device=dev)
        self.bmask = torch.as_tensor(self.xp.bmask, device=dev)
        # per-block (stage kernel) or per-job (march kernel) stage counts
        assert hc.march or hc.nblocks == self.xp.nblocks
        self.epoch = torch.zeros(hc.nblocks, dtype=torch.int32, device=dev)
        self.err = torch.zeros(4, dtype=torch.int32, device=dev)
        self.push = torch.as_tensor(self.xp.push, device=dev)
        self.cpush = torch.as_tensor(self.xp.cpush, device=dev)
        self.prime_src = torch.as_tensor(self.xp.prime_src, device=dev)
        self.prime_code = torch.as_tensor(self.xp.prime_code, device=dev)
        assert int(self.xp.push.max(initial=-1)) < e.plan.S
        assert self.prime_src.numel() == 0 or int(self.xp.prime_src.max()) < e.plan.S
        self.timeout_ticks = int(timeout_s * 1e8)
        self._distributed = distributed
        self.prime()

    def _agreed(self, err, distributed: bool) -> None:
        """All-ranks agreement after a local step that may have failed: every
        rank raises (after releasing what it holds) if any rank failed."""
        if not agree(err is None, distributed, self.e.device, self.group):
            self.close()
            raise err if err is not None else RuntimeError("xGMI setup failed on another rank")

    @staticmethod
    def _check_chain(integ) -> None:
        """The ring carries the ghosts of each stage's output to the next
        stage: every stage's halo input must be the previous stage's output."""
        st = integ.stages
        rot = integ.rotation
        for k in range(len(st)):
            prev = st[k - 1]
            q = st[k].Q
            out_prev = prev.out if k > 0 else [i for i in range(integ.nbuf) if rot[i] == prev.out][0]
            if q != out_prev:
                raise ValueError(f"integrator {integ.name}: stage {k} reads buffer {q}, not the previous output")

    # ---- descriptors --------------------------------------------------------
    def fill(self, d):
        from . import native
        d.xg = 1
        d.remote = 0
        d.blocks = 0
        d.nblocks = self.xp.nblocks
        d.ring = self.ring
        d.recv = self.base + CNT_BYTES
        d.push = native.ptr(self.push)
        d.cpush = native.ptr(self.cpush)
        d.peer_ring = native.ptr(self.peer_ring)
        d.peer_cnt = native.ptr(self.peer_cnt)
        d.cnt = self.base
        d.nprod = native.ptr(self.nprod)
        d.bmask = native.ptr(self.bmask)
        d.epoch = native.ptr(self.epoch)
        d.err = native.ptr(self.err)
        d.timeout_ticks = self.timeout_ticks
        return d

    # ---- initial / re-delivery ------------------------------------------------
    def prime(self) -> None:
        """Deliver the ghosts of the current state (pool[0]) into every peer's
        ring slot for the next stage.  Collective: all ranks, quiescent."""
        import torch.distributed as dist
        from . import native
        e = self.e
        torch.cuda.synchronize(e.device)
        ep = self.epoch
        e0 = int(ep[0].item())
        if not bool((ep == e0).all()):
            raise RuntimeError("xGMI epochs diverged across blocks")
        if dist.is_available() and dist.is_initialized() and self.world > 1:
            dist.barrier(group=self.group)   # nobody still reads the slot we are about to fill
        rc = self._lib.stsp_xg_prime_launch(native.dtype_code(e.dtype), native.ptr(e.pool[0]), e.plan.S,
                                            e.physics.F, native.ptr(self.prime_src), native.ptr(self.prime_code),
                                            int(self.prime_src.numel()), native.ptr(self.peer_ring), self.ring,
                                            e0, native.current_stream_handle())
        torch.cuda.synchronize(e.device)
        self._agreed(None if rc == 0 else RuntimeError(f"xGMI prime launch failed ({rc})"),
                     dist.is_available() and dist.is_initialized() and self.world > 1)
        if dist.is_available() and dist.is_initialized() and self.world > 1:
            dist.barrier(group=self.group)

    def check(self) -> None:
        if int(self.err[0].item()) != 0:
            raise RuntimeError("direct xGMI halo: a peer's ghosts did not arrive in time (poll timeout)")

    def close(self, collective: bool = True) -> None:
        """Explicit close: collective (every rank together, see IpcRing.close).
        The garbage-collection path passes ``collective=False``."""
        if getattr(self, "mem", None) is not None:
            self.mem.close(collective=collective)
        self.base = None

    def __del__(self):
        # a finalizer runs at a different point on every rank (reference
        # cycles, an exception unwinding on one rank): it must not join a
        # collective that could pair with an unrelated one
        try:
            self.close(collective=False)
        except Exception:
            pass


def agree(ok: bool, distributed: bool, device, group=None) -> bool:
    """All-ranks AND of a local success flag (True without a process group)."""
    if not distributed:
        return ok
    import torch.distributed as dist
    dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class IpcRing:
    """One uncached device allocation per rank, mapped by every peer through a
    dmabuf IPC handle exchanged over torch.distributed (``bases[p]``: rank p's
    allocation as seen from this process).  Every local step that can fail is
    followed by an all-ranks agreement, so all ranks raise together (after
    releasing what they hold) instead of leaving peers inside another
    collective."""

    def __init__(self, L, device, world: int, rank: int, peers, nbytes: int, group=None, cached: bool = False):
        """``cached``: ordinary device memory (``hipMalloc``) instead of an
        uncached ring, for payloads that are only read by a LATER kernel than
        the one that waited for them (the kernel boundary orders them); flags
        and tagged granules polled inside a kernel need the uncached ring."""
        import torch.distributed as dist
        self._lib = L
        self.cached = bool(cached)
        self.device = device
        self.group = group
        self.base = None
        self.opened: List[int] = []
        self.bases = {rank: 0}
        distributed = dist.is_available() and dist.is_initialized() and world > 1
        self.distributed = distributed
        if not distributed and any(p != rank for p in peers):
            raise RuntimeError("remote peers but no initialised torch.distributed group to exchange IPC handles")
        err = None
        off = 0
        hb = L.stsp_ipc_handle_bytes()
        h = (ctypes.c_char * hb)()
        try:
            base = ctypes.c_void_p()
            rc = (L.stsp_dev_alloc if self.cached else L.stsp_xg_alloc)(ctypes.c_size_t(nbytes), ctypes.byref(base))
            if rc != 0:
                raise RuntimeError(f"uncached allocation for the xGMI ring failed ({rc})")
            self.base = base.value
            self.bases[rank] = self.base
            if distributed:
                L.stsp_enable_peers(device.index if device.index is not None else torch.cuda.current_device())
                rc = L.stsp_ipc_get(ctypes.c_void_p(self.base), h)
                if rc != 0:
                    raise RuntimeError(f"hipIpcGetMemHandle failed ({rc})")
                off = int(L.stsp_ipc_offset(ctypes.c_void_p(self.base)))
                if off < 0:
                    raise RuntimeError("hipMemGetAddressRange failed on the ring")
        except RuntimeError as exc:
            err = exc
        self._agreed(err)
        if distributed:
            allh = [None] * world
            dist.all_gather_object(allh, (bytes(h), off), group=group)
            try:
                for p in peers:
                    if p == rank:
                        continue
                    ptr = ctypes.c_void_p()
                    hp, offp = allh[p]
                    rc = L.stsp_ipc_open((ctypes.c_char * hb).from_buffer_copy(hp), ctypes.byref(ptr))
                    if rc != 0:
                        raise RuntimeError(f"hipIpcOpenMemHandle of rank {p} failed ({rc})")
                    self.opened.append(ptr.value)
                    self.bases[p] = ptr.value + offp       # the mapping opens at the allocation's base
            except RuntimeError as exc:
                err = exc
            self._agreed(err)

    def _agreed(self, err) -> None:
        if not agree(err is None, self.distributed, self.device, self.group):
            self.close()
            raise err if err is not None else RuntimeError("xGMI setup failed on another rank")

    def close(self, collective: bool = True) -> None:
        """Collective when distributed (every rank closes its ring together,
        as every explicit call site does).  Order: this rank's kernels are done
        (no more stores into peers' rings), its peer mappings are closed, then a
        group barrier, and only then does the ring go back to the process's
        pool, where the next ``stsp_xg_alloc`` zeroes and reuses it: without the
        barrier a peer still inside its last launch could store tagged granules
        into a ring this rank had already handed to a new exchange.

        ``collective=False`` (finalizers): no barrier, and the
        allocation is NOT handed back (neither to the pool nor to the driver),
        since a peer may still store into it; it stays with the process."""
        import torch.distributed as dist
        if getattr(self, "_closed", False):
            return
        self._closed = True
        L = self._lib
        if self.base or self.opened:
            torch.cuda.synchronize(self.device)
        for p in self.opened:
            L.stsp_ipc_close(ctypes.c_void_p(p))
        self.opened = []
        if not collective and self.distributed:
            self.base = None                     # leaked on purpose: a peer may still store into it
            return
        if self.distributed and dist.is_initialized():
            dist.barrier(group=self.group)       # every rank, with or without a ring
        if self.base:
            if self.cached:
                L.stsp_dev_free(ctypes.c_void_p(self.base))
            else:
                L.stsp_xg_free(ctypes.c_void_p(self.base))     # back to the process's ring pool
            self.base = None


def _declare(L):
    vp, ci = ctypes.c_void_p, ctypes.c_int
    L.stsp_xg_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
    L.stsp_xg_alloc.restype = ci
    L.stsp_xg_free.argtypes = [vp]
    L.stsp_xg_free.restype = ci
    L.stsp_dev_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
    L.stsp_dev_alloc.restype = ci
    L.stsp_dev_free.argtypes = [vp]
    L.stsp_dev_free.restype = ci
    L.stsp_xg_pool.argtypes = [ctypes.POINTER(ctypes.c_longlong)]
    L.stsp_xg_pool.restype = ci
    L.stsp_ipc_handle_bytes.argtypes = []
    L.stsp_ipc_handle_bytes.restype = ci
    L.stsp_ipc_get.argtypes = [vp, vp]
    L.stsp_ipc_get.restype = ci
    L.stsp_ipc_offset.argtypes = [vp]
    L.stsp_ipc_offset.restype = ctypes.c_longlong
    L.stsp_ipc_open.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p)]
    L.stsp_ipc_open.restype = ci
    L.stsp_ipc_close.argtypes = [vp]
    L.stsp_ipc_close.restype = ci
    L.stsp_enable_peers.argtypes = [ci]
    L.stsp_enable_peers.restype = ci
    L.stsp_xg_prime_launch.argtypes = [ci, vp, ci, ci, vp, vp, ci, vp, ci, ci, vp]
    L.stsp_xg_prime_launch.restype = ci
    L.stsp_xg_protocol.argtypes = []
    L.stsp_xg_protocol.restype = ci
    L.stsp_xg_slots.argtypes = []
    L.stsp_xg_slots.restype = ci
    return L
