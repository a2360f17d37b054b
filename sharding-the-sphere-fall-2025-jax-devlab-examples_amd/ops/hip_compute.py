"""HIP stage computation for ``Engine(backend='hip')``: one fused gfx950 kernel
launch per RK stage (two when the rank has remote neighbours: interior blocks
while the halo messages fly, boundary blocks after).  The launch replaces the
reference's XLA-generated halo ops (extract / reverse / ``.at[].set``,
PY:166-197) and its numerics (PDF s.4, s.19: FV-PLR, 870 flops per cell).

All shape contracts the kernel relies on are checked here, on the host, once,
before anything is launched (a bad index in a hand-written kernel can reset a
whole node).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import native
from ..models.integrators import Stage

BLOCK_SHAPES = ((16, 16), (32, 8), (16, 8), (8, 16), (8, 8))
# The streaming stage (ops/csrc/march_kernel.hip): (64, R) = one wave marches 60
# columns up R rows of a tile.  Shallow water with a PLR limiter; remote ghosts
# only through the direct xGMI exchange (XgmiHalo switches a rank to it,
# rows 4), never through RCCL's receive buffer and block lists.
MARCH_SHAPES = ((64, 4), (64, 8), (64, 16), (64, 32))


MARCH_AUTO = (64, 4)
MARCH_CELLS_PER_CU = 8192


def march_supported(phys_id: int, limiter: int, remote: bool, xgmi: bool = False) -> bool:
    return phys_id == 2 and limiter != 4 and (not remote or xgmi)


def march_tables(engine) -> dict:
    """Compact-geometry tables of the streaming stage (march_kernel.hip, CG):
    tile origins, the panel-shared geometry of the fused step
    (ops/fused.py::kernel_geometry: 1/A, curvature sum and centre per
    panel-local cell, edge lengths, panel frames) and the topography b in the
    padded state layout with its ghost ring filled through the same-rank halo
    map (None without topography)."""
    from .fused import kernel_geometry
    e = engine
    plan, lay = e.plan, e.layout
    kg = kernel_geometry(lay, e.grid)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=e.dtype, device=e.device)
    torg = np.array([lay.tile_origin(tid) for tid in plan.tiles], dtype=np.int32).reshape(-1, 3)
    out = {"torg": torch.as_tensor(torg, device=e.device), "crec": t(kg["crec"]), "lxt": t(kg["lxt"]),
           "frames": [int(v) for v in kg["frames"]], "bpad": None}
    gf = getattr(e.physics, "global_fields", None)
    if gf is not None:
        b = np.asarray(gf(e.grid)[2], dtype=np.float64)
        if np.any(b != 0):
            from ..parallel.layout import ghost_xy
            n, P, ng = plan.n, plan.P, plan.ng
            bp = np.zeros((plan.T, P, P))
            for li, tid in enumerate(plan.tiles):
                f, I0, J0 = lay.tile_origin(tid)
                bp[li, ng:ng + n, ng:ng + n] = b[f, J0:J0 + n, I0:I0 + n]
            # every edge ghost from its global source (same-rank and remote alike:
            # the topography is static, so no exchange carries it)
            gs = lay.ghost_sources(e.rank)                       # [T, 4, ng, n]
            bg = b.reshape(-1)
            pos = np.arange(n)
            for li in range(plan.T):
                for side in range(4):
                    for k in range(ng):
                        x, y = ghost_xy(side, k, pos, n)
                        bp[li, y + ng, x + ng] = bg[gs[li, side, k]]
            out["bpad"] = t(bp.reshape(-1))
    return out


def block_threads_formula(bx: int, by: int, w10: bool = True) -> int:
    """Threads of a stage block: one per x- and y-edge, rounded to wave64;
    256-cell blocks with at most 544 edges run the ten-wave role map
    (stage_kernel.hip, Geom::W10; off in the ``w9`` library variant)."""
    ne = (bx + 1) * by + bx * (by + 1)
    if w10 and bx * by == 256 and ne <= 544:
        return 640
    return (ne + 63) // 64 * 64


_NT_CACHE = {}


def block_threads(bx: int, by: int) -> int:
    """Threads per stage block of the library that is (or would be) loaded:
    ``stsp_block_threads`` (Geom<BX, BY>::NT as compiled) when the library is
    present, else the formula for the selected build variant."""
    key = (bx, by)
    if key not in _NT_CACHE:
        nt = -1
        try:
            L = native.load(build_if_missing=False)
            L.stsp_block_threads.argtypes = [ctypes.c_int, ctypes.c_int]
            L.stsp_block_threads.restype = ctypes.c_int
            nt = int(L.stsp_block_threads(bx, by))
        except (OSError, AttributeError):
            nt = -1
        if nt <= 0:
            import os
            nt = block_threads_formula(bx, by, w10=os.environ.get("STSP_VARIANT", "") != "w9")
        _NT_CACHE[key] = nt
    return _NT_CACHE[key]


def block_supports(bx: int, by: int, limiter: int) -> bool:
    """PPM (limiter 4) loads its 3-layer window one cell per thread."""
    return limiter != 4 or (bx + 6) * (by + 6) <= block_threads(bx, by)


def choose_block(n: int, tiles: int = 0, cus: int = 0, limiter: int = 0, esize: int = 8):
    """Block shape for a rank holding ``tiles`` tiles of ``n x n`` cells
    (``esize``: bytes per value, 8 = fp64, 4 = fp32).

    One pass (the 16x16 grid fits the ``cus`` compute units): a block's
    critical path is its memory round trips plus its flux and update chains,
    and the issue part scales with the waves a block puts on each SIMD, so the
    smallest shape that still fits in one pass wins.  Measured at C96 / t=2
    (tools/small_grid_probe.sh, profiles/r1_small_grid_block_shapes_v4.txt):
    3 tiles of 48^2 take 4.40 us per stage with 16x16 and 3.67 us with 8x8;
    12 tiles 4.67 us with 16x16 and 4.05 us with 16x8; the full 24 tiles
    (216 blocks) 4.86 us with 16x16 and 5.02-5.12 us with the smaller shapes.

    Several passes: the CU hides one block's round trips and barriers behind
    other resident blocks, and small blocks (16x8: 5 waves, 8x8: 3 waves) keep
    more of them in flight than 16x16 (10 waves, 3 blocks = 30 of 32 wave
    slots).  Measured per stage (profiles/r1_block_shapes_by_size.txt):
    fp32 16x8 is best from C128 up (C720: 83.6 us vs 103.7 for 16x16);
    fp64 16x8 up to about 8 blocks of 16x8 per CU (C180: 12.4 vs 13.8 us),
    8x8 beyond (C256: 20.2 vs 23.8, C720: 141 vs 196 us).  Shapes that cannot
    run ``limiter`` (8x8 with PPM) are skipped.
    """
    def count(bx, by):
        return tiles * -(-n // bx) * -(-n // by)

    def waste(bx, by):
        return -(-n // bx) * -(-n // by) * bx * by - n * n

    if tiles and cus:
        if count(16, 16) <= cus:
            fits = [(bx * by, waste(bx, by), count(bx, by), -bx, (bx, by)) for bx, by in BLOCK_SHAPES
                    if count(bx, by) <= cus and bx * by < 256 and block_supports(bx, by, limiter)]
            if fits:
                return min(fits)[-1]   # ties: the wider (contiguous-row) block
            return (16, 16)
        if esize >= 8 and count(16, 8) > 8 * cus and block_supports(8, 8, limiter):
            return (8, 8)
        return (16, 8)
    best, w0 = (16, 16), None
    for bx, by in BLOCK_SHAPES:
        if bx * by != 256:
            continue
        w = waste(bx, by)
        if w0 is None or w < w0:
            best, w0 = (bx, by), w
    return best


class HipCompute:
    def __init__(self, engine):
        e = engine
        self.e = e
        self.lib = native.require_native()
        if e.device.type != "cuda":
            raise RuntimeError("backend='hip' needs a GPU tensor device")
        plan = e.plan
        phys = e.physics
        self.phys_id = phys.kernel_id
        self.dcode = native.dtype_code(e.dtype)
        n, T = plan.n, plan.T
        self.march_wanted = False       # the size rule picks the streaming stage (XgmiHalo may switch)
        if e.block is None:
            cus = torch.cuda.get_device_properties(e.device).multi_processor_count
            bx, by = choose_block(n, T, cus, getattr(phys, "limiter", 0), torch.tensor([], dtype=e.dtype).element_size())
            # streaming stage once the rank streams: measured C720 (3.1M cells, 12k per CU)
            # fp64 423 vs 467 us/step, fp32 190 vs 252 (64 x 4; 64 x 8: 431 / 203); C360 (3k per CU) a tie,
            # C180 the block kernel (43 vs 75): too few marches to hide their latency
            lim = int(phys.kernel_params().get("limiter", 0))
            self.march_wanted = march_supported(self.phys_id, lim, False) and T * n * n >= MARCH_CELLS_PER_CU * cus
            if self.march_wanted and march_supported(self.phys_id, lim, plan.num_recv > 0):
                bx, by = MARCH_AUTO
        else:
            bx, by = e.block
        self.march = (bx, by) in MARCH_SHAPES
        if self.march:
            if not march_supported(self.phys_id, int(phys.kernel_params().get("limiter", 0)), False) or \
                    (plan.num_recv > 0 and by != 4):
                raise ValueError("the streaming stage (block (64, R)) runs shallow water with a PLR limiter; "
                                 "a rank with remote ghosts marches 4 rows per wave through the xGMI exchange")
        elif (bx, by) not in BLOCK_SHAPES:
            raise ValueError(f"unsupported block shape {(bx, by)}")
        self._shape(bx, by)
        # streaming stage geometry: compact (panel-shared tables, grad b from b) for fp64,
        # per-tile records for fp32 (C720 64x4: fp64 409 vs 415 us/step, fp32 225 vs 195,
        # where the compact path spills; profiles/r3_march/sizes_compact_geometry_ab.log);
        # STSP_MARCH_COMPACT=0/1 overrides
        self._tables()
        t = e.tens
        F, S = phys.F, plan.S
        # ---- host-side shape contract checks ----------------------------
        for b in e.pool:
            assert b.shape == (F, S) and b.is_contiguous() and b.dtype == e.dtype
        assert e.gmap.dtype == torch.int32 and e.gmap.shape == (T, 4, plan.ng, n)
        assert phys.halo <= plan.ng
        assert t["invA"].shape == (T, n, n)
        assert t["ex"].shape == (T, n, n + 1) and t["ey"].shape == (T, n + 1, n)
        if "pedge" in t:
            assert t["pedge"].dtype == torch.int32 and t["pedge"].shape == (T,)
        if "pe_base" in t:      # panel-edge ghost interpolation tables (models/base.py)
            assert t["pe_base"].dtype == torch.int32 and t["pe_base"].shape == (T, 4, 3, n)
            assert t["pe_t"].dtype == e.dtype and t["pe_t"].shape == (T, 4, 3, n)
            # pairs chosen on the whole panel edge: tile-local b leaves [0, n-2] by
            # up to layer + 1 cells, into the carried corner ghosts (models/base.py)
            assert int(t["pe_base"].min()) >= -3 and int(t["pe_base"].max()) <= n + 1
            # the kernel reads the interpolation pair (b, b + 1) of ghost layer k < KG
            # from the block's window: -NG <= b - j <= NG - 1 for strip cell j
            # (PLR: NG = 2, one layer; PPM: NG = 3, two layers)
            ppm = int(phys.kernel_params().get("limiter", 0)) == 4
            ng_k, kg = (3, 2) if ppm else (2, 1)
            off = t["pe_base"][:, :, :kg].long() - torch.arange(n, device=t["pe_base"].device)
            assert int(off.min()) >= -ng_k and int(off.max()) <= ng_k - 1, \
                "panel-edge interpolation pair outside the block window"
        if self.phys_id == 2:
            assert t["mx"].shape == (T, 3, n + 1) and t["my"].shape == (T, 3, n + 1)
            assert t["cgeo"].shape == (T, n, n, 8)
        assert S == T * (n + 2 * plan.ng) ** 2
        pm = plan.push_map
        assert pm.shape == (T, 4, plan.ng, n) and pm.max(initial=-1) < S
        self.push = torch.as_tensor(pm, dtype=torch.int32, device=e.device)
        # carried tile-corner ghosts: pushed by their own table, remote ones read through corner_map
        cpm, cgm = plan.corner_push, plan.corner_map
        assert cpm.shape == cgm.shape == (T, 4, plan.ng, plan.ng) and cpm.max(initial=-1) < S and cgm.max() < S
        assert plan.corner_carried.sum() == 0 or n >= 2 * plan.ng
        assert (-1 - cgm[cgm < 0]).max(initial=-1) < plan.num_recv
        self.cpush = torch.as_tensor(cpm, dtype=torch.int32, device=e.device)
        self.cgmap = torch.as_tensor(cgm, dtype=torch.int32, device=e.device)
        recv = e.transport.recv
        assert recv.shape == (plan.num_recv, F)
        gm = plan.ghost_map
        if gm.size:
            assert gm.max() < S and (-1 - gm[gm < 0]).max(initial=-1) < plan.num_recv
        for k in t:
            t[k] = t[k].contiguous()
        self.remote = plan.num_recv > 0
        if self.remote:
            inter, bnd = plan.block_classes(bx, by)
            self.blk_interior = torch.as_tensor(inter, dtype=torch.int32, device=e.device)
            self.blk_boundary = torch.as_tensor(bnd, dtype=torch.int32, device=e.device)
            assert (inter.size == 0 or inter.max() < self.nblocks) and (bnd.size == 0 or bnd.max() < self.nblocks)
        self._g = phys.kernel_params().get("g", 0.0)
        self._omega2 = phys.kernel_params().get("omega2", 0.0)
        self._lim = int(phys.kernel_params().get("limiter", 0))

    def _shape(self, bx: int, by: int) -> None:
        n, T = self.e.plan.n, self.e.plan.T
        self.bx, self.by = bx, by
        self.march = (bx, by) in MARCH_SHAPES
        if self.march:   # jobs: (tile, 60-column strip, R-row segment), four per workgroup
            self.nbx, self.nby = -(-n // 60), -(-n // by)
        else:
            self.nbx, self.nby = -(-n // bx), -(-n // by)
        self.nblocks = T * self.nbx * self.nby

    def _tables(self) -> None:
        import os
        e = self.e
        cg = os.environ.get("STSP_MARCH_COMPACT", "1" if e.dtype == torch.float64 else "0") != "0"
        self.mt = march_tables(e) if self.march and cg else None

    def use_march_with_xgmi(self) -> bool:
        """Switch a rank with remote ghosts to the streaming stage when the size
        rule wants it: the direct xGMI exchange (XgmiHalo) delivers its remote
        ghosts inside the march kernel (rows 4).  True if the rank marches."""
        if self.march:
            return True
        if not self.march_wanted or self.e.block is not None:
            return False
        self._shape(*MARCH_AUTO)
        self._tables()
        # the interior / boundary block lists describe the old block grid: a
        # march job id is not a block id, so the split launch path is closed for
        # this engine (its stages run inside the xGMI stage ops)
        self.blk_interior = self.blk_boundary = None
        self._xg_march = True
        return True

    def desc(self, st: Stage, dt: float, blocks: Optional[torch.Tensor], nblocks: int,
             remote: bool = False) -> native.StageDesc:
        e = self.e
        t = e.tens
        p = native.ptr
        d = native.StageDesc()
        d.X = p(e.pool[st.X])
        d.Q = p(e.pool[st.Q])
        d.acc_in = p(e.pool[st.acc_in]) if st.acc_in >= 0 else 0
        d.out = p(e.pool[st.out])
        d.acc_out = p(e.pool[st.acc_out]) if st.acc_out >= 0 else 0
        d.recv = p(e.transport.recv) if e.transport.recv.numel() else 0
        d.gmap = p(e.gmap)
        d.push = p(self.push)
        d.cpush = p(self.cpush)
        d.cgmap = p(self.cgmap)
        d.blocks = p(blocks) if blocks is not None else 0
        d.invA = p(t["invA"])
        d.ex = p(t["ex"])
        d.ey = p(t["ey"])
        if self.phys_id == 2:
            d.mx, d.my, d.cgeo = p(t["mx"]), p(t["my"]), p(t["cgeo"])
        if "pedge" in t:
            d.pedge = p(t["pedge"])
        if "pe_base" in t:
            d.pe_base, d.pe_t = p(t["pe_base"]), p(t["pe_t"])
        if self.mt is not None:
            mt = self.mt
            d.torg, d.crec, d.lxt = p(mt["torg"]), p(mt["crec"]), p(mt["lxt"])
            d.bpad = p(mt["bpad"]) if mt["bpad"] is not None else 0
            d.Nf = e.layout.N
            for f in range(6):
                d.frames[f] = mt["frames"][f]
        d.ntile = e.plan.T
        d.n = e.plan.n
        d.S = e.plan.S
        d.mg = e.plan.ng
        d.pw = e.plan.P
        d.nblocks = nblocks
        d.limiter = self._lim
        d.remote = 1 if remote else 0
        d.a0, d.a1, d.a2 = st.a0, st.a1, st.a2
        d.c0, d.c1, d.c2 = st.c0, st.c1, st.c2
        d.dt = dt
        d.g = self._g
        d.omega2 = self._omega2
        return d

    def launch(self, d: native.StageDesc, stream: Optional[int] = None) -> None:
        rc = self.lib.stsp_stage_launch(self.phys_id, self.dcode, self.bx, self.by, d,
                                        native.current_stream_handle() if stream is None else stream)
        native.check(rc, "stage kernel")

    def stage(self, st: Stage, dt: float, recv, part: str = "all") -> None:
        if getattr(self, "_xg_march", False):
            raise RuntimeError("this engine marches with the direct xGMI exchange: its stages run through "
                               "XgmiHalo (the interior / boundary split has no march form)")
        if not self.remote:
            if part in ("all", "interior"):
                self.launch(self.desc(st, dt, None, self.nblocks))
            return
        if part in ("all", "interior") and self.blk_interior.numel():
            self.launch(self.desc(st, dt, self.blk_interior, self.blk_interior.numel()))
        if part in ("all", "boundary") and self.blk_boundary.numel():
            self.launch(self.desc(st, dt, self.blk_boundary, self.blk_boundary.numel(), remote=True))
