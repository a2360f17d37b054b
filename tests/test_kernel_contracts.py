"""Host-side contracts of the gfx950 stage kernel that can be checked without a
GPU: the ten-wave role tables of 256-cell blocks (ops/csrc/stage_kernel.hip,
Geom::OWN_TAB / FLUX_TAB / RING_TAB in stage_common.h) must give every own cell, every edge and
every window-ring cell exactly one thread."""
import os
import re

import pytest

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "sharding-the-sphere-fall-2025-jax-devlab-examples_amd", "ops", "csrc", "stage_common.h")


def _tables():
    s = open(SRC).read()
    out = {}
    for name in ("OWN_TAB", "FLUX_TAB", "RING_TAB"):
        v = int(re.search(name + r" = (0x[0-9a-f]+)ULL", s).group(1), 16)
        out[name] = [(v >> (4 * w)) & 15 for w in range(10)]
    return out


@pytest.mark.parametrize("bx,by,ng", [(16, 16, 2), (16, 16, 3)])
def test_ten_wave_role_tables_cover_block(bx, by, ng):
    t = _tables()
    own, flux, ring = t["OWN_TAB"], t["FLUX_TAB"], t["RING_TAB"]
    nin, ne = bx * by, (bx + 1) * by + bx * (by + 1)
    ring_cells = (bx + 2 * ng) * (by + 2 * ng) - nin
    lanes = range(64)
    own_ids = sorted(o * 64 + l for o in own if o != 15 for l in lanes)
    assert own_ids == list(range(nin))                       # every own cell once
    edge_ids = sorted(f * 64 + l for f in flux if f != 15 for l in lanes if f * 64 + l < ne)
    assert edge_ids == list(range(ne))                       # every edge once
    ring_ids = sorted(r * 64 + l for w, r in enumerate(ring) if r != 15 for l in lanes)
    assert ring_ids[:ring_cells] == list(range(ring_cells))  # every ring cell once
    assert all(own[w] == 15 for w, r in enumerate(ring) if r != 15)   # ring only on waves without own cells
    # SIMD balance (wave w runs on SIMD w % 4): nine flux iterations, no own-cell
    # wave on the SIMD that runs three of them
    iters = [sum(1 for w in range(10) if w % 4 == s and flux[w] != 15) for s in range(4)]
    owns = [sum(1 for w in range(10) if w % 4 == s and own[w] != 15) for s in range(4)]
    assert sum(iters) == -(-ne // 64) and max(iters) == 3
    assert all(owns[s] == 0 for s in range(4) if iters[s] == 3)


def test_block_threads_matches_library():
    """The host's thread count (used by the PPM window check and the launch
    geometry) equals Geom<BX, BY>::NT of the library as built."""
    import ctypes
    from stsphere.ops import build as b
    from stsphere.ops.hip_compute import BLOCK_SHAPES, block_threads, block_threads_formula
    if not os.path.exists(b.lib_for("")):
        pytest.skip("library not built")
    L = ctypes.CDLL(b.lib_for(""), mode=ctypes.RTLD_GLOBAL)
    L.stsp_block_threads.argtypes = [ctypes.c_int, ctypes.c_int]
    for bx, by in BLOCK_SHAPES:
        nt = L.stsp_block_threads(bx, by)
        assert nt == block_threads(bx, by) == block_threads_formula(bx, by)
    assert L.stsp_block_threads(7, 7) == -1
    assert block_threads_formula(16, 16, w10=False) == 576


def _edge_of_slot(slot, lane, bx=16, by=16, sx=7, sy=5):
    """Python mirror of stage_common.h::edge_of_slot (border-edge flux slots)."""
    nx, ny = (bx + 1) * by, bx * (by + 1)
    ix, iy = bx - 3, by - 3
    q, u4 = lane & 3, lane >> 2
    b = q if q < 2 else q + (bx - 3)
    if slot == sx:
        return u4 * (bx + 1) + b
    if slot == sy:
        return nx + b * bx + u4
    u = (slot - (slot > sy) - (slot > sx)) * 64 + lane
    if u < by * ix:
        r = u // ix
        return r * (bx + 1) + 2 + (u - r * ix)
    v = u - by * ix
    if v < iy * bx:
        r = v // bx
        return nx + (2 + r) * bx + (v - r * bx)
    return nx + ny


def test_border_edge_slots_are_a_bijection():
    """The PEW edge layout (panel-edge fix-up inside the border-edge waves)
    gives every edge of a 16x16 block exactly one lane of the nine flux slots;
    slot 7 holds exactly the x-edges at columns 0, 1, 15, 16 and slot 5 the
    y-edges at rows 0, 1, 15, 16, on waves of SIMDs 3 and 2."""
    bx = by = 16
    nx, ny = (bx + 1) * by, bx * (by + 1)
    t = _tables()
    slots = [f for f in t["FLUX_TAB"] if f != 15]
    assert sorted(slots) == list(range(9))
    ids = [_edge_of_slot(s, l) for s in slots for l in range(64)]
    real = sorted(i for i in ids if i < nx + ny)
    assert real == list(range(nx + ny))
    src = open(SRC).read()
    assert "constexpr int PEW_SX = 7, PEW_SY = 5;" in src
    flux = t["FLUX_TAB"]
    assert flux.index(7) % 4 == 3 and flux.index(5) % 4 == 2
    s0 = {_edge_of_slot(7, l) for l in range(64)}
    assert s0 == {r * (bx + 1) + c for r in range(by) for c in (0, 1, bx - 1, bx)}
    s1 = {_edge_of_slot(5, l) for l in range(64)}
    assert s1 == {nx + r * bx + c for r in (0, 1, by - 1, by) for c in range(bx)}


def test_rccl_resolved_from_the_loaded_library_and_version_checked():
    """The runtime does not link RCCL: it resolves the calls it uses from the
    librccl.so.1 the process already holds (PyTorch's copy), so the library it
    runs is the one PyTorch reports, and its version is checked against the
    API range csrc/rccl_abi.h declares (round-3 verdict: headers 2.27.7 vs
    the loaded 2.26.6)."""
    import torch
    from stsphere.ops import build as b
    from stsphere.ops.native_runtime import rccl_version
    v = rccl_version()
    major, minor, patch = torch.cuda.nccl.version()
    assert v == major * 10000 + minor * 100 + patch
    assert 21800 <= v <= 22999
    # no DT_NEEDED entry for librccl in the in-tree library
    import shutil
    import subprocess
    tool = shutil.which("llvm-readelf") or "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not os.path.exists(tool):
        pytest.skip("llvm-readelf not available")
    dyn = subprocess.run([tool, "-d", b.lib_for("")], capture_output=True, text=True, check=True).stdout
    needed = [ln for ln in dyn.splitlines() if "(NEEDED)" in ln]
    assert needed and not any("rccl" in ln for ln in needed), needed
