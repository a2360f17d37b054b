#!/usr/bin/env python
"""Stage-kernel probe (GPU): per-launch time of the fused stage kernel in a
captured graph (production library), and per-phase shares from the in-kernel
stamp build (``STSP_VARIANT=diag``; shares only, never its run time).

    python tools/kprobe.py [--N 96] [--t 2] [--dtype fp64] [--phys swe]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--t", type=int, default=2)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--phys", default="swe")
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--blocks", default="16x16,16x8,8x16,32x8,8x8")
    ap.add_argument("--limit", type=int, default=0, help="launch only this many blocks (latency probe)")
    ap.add_argument("--no-pedge", action="store_true",
                    help="timing only: clear the panel-edge bits (no ghost interpolation; wrong numerics)")
    a = ap.parse_args()
    if a.stamps and not os.environ.get("STSP_VARIANT", "").startswith("diag"):
        os.environ["STSP_VARIANT"] = "diag"
    import torch
    from stsphere.engine import Engine
    from stsphere.models.advection import Advection
    from stsphere.models.diffusion import Diffusion
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops import native
    from stsphere.parallel.layout import TileLayout

    dtype = torch.float64 if a.dtype == "fp64" else torch.float32
    mk = {"swe": lambda: ShallowWater("tc5"), "adv": lambda: Advection(), "diff": lambda: Diffusion()}[a.phys]
    grid = CubedSphereGrid(a.N)
    L = TileLayout(a.N, a.t, 1, ng=2)
    res = {"N": a.N, "t": a.t, "dtype": a.dtype, "phys": a.phys, "no_pedge": a.no_pedge}
    for bs in a.blocks.split(","):
        bx, by = map(int, bs.split("x"))
        e = Engine(mk(), L, grid=grid, dtype=dtype, device="cuda", backend="hip", block=(bx, by))
        hc = e.compute
        if a.no_pedge and "pedge" in e.tens:
            e.tens["pedge"].zero_()
        hc.bx, hc.by = bx, by
        hc.nbx, hc.nby = -(-L.n // bx), -(-L.n // by)
        hc.nblocks = e.plan.T * hc.nbx * hc.nby
        st = e.integ.stages[1]
        d = hc.desc(st, e.dt, None, hc.nblocks)
        if a.limit:
            # first `limit` logical blocks through an explicit work list (no XCD remap)
            lst = torch.arange(a.limit, dtype=torch.int32, device="cuda")
            d = hc.desc(st, e.dt, lst, a.limit)
        stamps = None
        if a.stamps:
            stamps = torch.zeros(hc.nblocks * 16 * 16, dtype=torch.int64, device="cuda")
            d.stamps = native.ptr(stamps)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(5):
                hc.launch(d)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(a.reps):
                hc.launch(d)
        g.replay()
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(3):
            g.replay()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1e3 / (3 * a.reps)
        r = {"us_per_launch": us, "nblocks": hc.nblocks}
        if a.stamps:
            import numpy as np
            ne = (bx + 1) * by + bx * (by + 1)
            nw = 10 if (bx * by == 256 and ne <= 544 and os.environ.get("STSP_W9") != "1") else -(-ne // 64)   # waves per block
            st_ = stamps.view(-1, 16, 16).cpu().numpy().astype("float64")[:, :nw]   # [block, wave, k]
            t0_ = st_[:, :, 0].min(axis=1)                         # block start (first wave)
            rel = st_ - t0_[:, None, None]
            names = ["start", "prefetch", "window", "barrier1", "faces+barrier", "flux", "end", "barrier2",
                     "update_computed", "out_stored", "pushes_stored", "pe_fixup"]
            # median over blocks of each wave's time at each stamp, relative to block start
            r["wave_stamp_cycles_median"] = {names[k]: [float(np.median(rel[:, w, k])) for w in range(nw)]
                                             for k in range(len(names))}
            tot = st_[:, :, 6].max(axis=1) - t0_
            r["block_cycles_median"] = float(np.median(tot))
            r["block_cycles_max"] = float(tot.max())
        res[bs] = r
    # launch floor: a 1-element indexed-copy kernel, same graph method
    src = torch.zeros(8, dtype=dtype, device="cuda")
    idx = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        native.copy_index(src, idx, src, idx, 1, 0, 0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(a.reps):
            native.copy_index(src, idx, src, idx, 1, 0, 0)
    g.replay()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(3):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    res["tiny_kernel_us_per_launch"] = t0.elapsed_time(t1) * 1e3 / (3 * a.reps)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
