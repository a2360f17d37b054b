#!/usr/bin/env python
"""Fused-step probe: launch time (eager, back to back; and graph replay) and
per-phase wave-0 stamps of every block (prologue, faces / updates of each
stage), split into panel-edge and interior blocks.  One JSON line.

    python tools/fused_probe.py --N 96 --t 2 --reps 50 --stamps
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=96)
    ap.add_argument("--t", type=int, default=2)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--stage", action="store_true", help="also time the launch-per-stage step")
    ap.add_argument("--B", type=int, default=0, help="block size (0: the residency-aware choice)")
    ap.add_argument("--loopback", action="store_true",
                    help="every other tile's window cells through the rank's own xGMI ring (tagged granules)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.fused import FusedKernel
    from stsphere.ops.native_runtime import NativeStepper
    from stsphere.parallel.layout import TileLayout
    dt = torch.float64 if a.dtype == "fp64" else torch.float32
    L = TileLayout(a.N, a.t, 1, ng=2, loopback=a.loopback)
    e = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(a.N), dtype=dt, device="cuda", backend="hip")
    fk = FusedKernel(e, B=a.B or None)
    out = {"N": a.N, "t": a.t, "dtype": a.dtype, "blocks": fk.plan.nb, "B": fk.plan.B, "loopback": a.loopback}
    fk.step(4)
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(a.reps):
        fk.launch(0)
        fk.launch(1)
    s1.record()
    torch.cuda.synchronize()
    out["eager_us_per_step"] = s0.elapsed_time(s1) * 1e3 / (2 * a.reps)
    r = NativeStepper(e, use_graph=True, steps_per_graph=2 * a.reps, fused=fk)
    r.prepare(2 * a.reps)
    r.run(2 * a.reps)
    torch.cuda.synchronize()
    s0.record()
    r.run(2 * a.reps)
    s1.record()
    torch.cuda.synchronize()
    out["graph_us_per_step"] = s0.elapsed_time(s1) * 1e3 / (2 * a.reps)
    for spl in (20, 2 * a.reps):
        r3 = NativeStepper(e, use_graph=True, steps_per_graph=2 * a.reps, fused=fk, steps_per_launch=spl)
        r3.prepare(2 * a.reps)
        r3.run(2 * a.reps)
        torch.cuda.synchronize()
        s0.record()
        r3.run(2 * a.reps)
        s1.record()
        torch.cuda.synchronize()
        fk.check()
        out[f"multi{spl}_us_per_step"] = s0.elapsed_time(s1) * 1e3 / (2 * a.reps)
        r3.close()
    # host-timed single runs of 20 steps, like bench.py's timed region
    import time
    r4 = NativeStepper(e, use_graph=True, steps_per_graph=20, fused=fk, steps_per_launch=20)
    r4.prepare(20)
    host = {"graph": [], "direct": []}
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r4.run(20)
        torch.cuda.synchronize()
        host["graph"].append((time.perf_counter() - t0) * 1e6 / 20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fk.launch(0, nsteps=20)
        torch.cuda.synchronize()
        host["direct"].append((time.perf_counter() - t0) * 1e6 / 20)
    r4.close()
    out["host_timed_20_us_per_step"] = {k: round(min(v), 3) for k, v in host.items()}
    if a.stage:
        e2 = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(a.N), dtype=dt, device="cuda", backend="hip")
        r2 = NativeStepper(e2, use_graph=True, steps_per_graph=2 * a.reps)
        r2.prepare(2 * a.reps)
        r2.run(2 * a.reps)
        torch.cuda.synchronize()
        s0.record()
        r2.run(2 * a.reps)
        s1.record()
        torch.cuda.synchronize()
        out["stage_graph_us_per_step"] = s0.elapsed_time(s1) * 1e3 / (2 * a.reps)
    if a.stamps:
        nb = fk.plan.nb
        FW = 32                              # stamp row width (fused_step.hip FST_W)
        st = torch.zeros((nb, 16, FW), dtype=torch.int64, device="cuda")
        for d in fk.descs:
            d.stamps = st.data_ptr()
        for _ in range(3):
            fk.launch(0)
        torch.cuda.synchronize()
        raw = st.cpu().numpy()
        v = raw[:, :, :16].astype(np.float64)
        for d in fk.descs:
            d.stamps = 0
        # placement: HW_ID (SIMD bits 5:4, CU 11:8, SH 12, SE 15:13) and XCC_ID per wave
        hw, xcc, disp = raw[:, :, 16], raw[:, :, 17], raw[:, :, 18]
        live = v[:, :, 0] != 0
        simd = (hw >> 4) & 3
        blk_xcc = np.array([int(xcc[b][live[b]][0]) & 15 for b in range(nb)])
        blk_disp = np.array([int(disp[b][live[b]][0]) for b in range(nb)])
        # waves of one block sharing a SIMD: is it always w mod 4?
        grp_ok = all(len(set(int(simd[b, w]) for w in range(16) if live[b, w] and w % 4 == r)) == 1
                     for b in range(nb) for r in range(4))
        out["placement"] = {
            "simd_of_wave_mod4_consistent": bool(grp_ok),
            "simd_order_block0": [int(simd[0, w]) for w in range(16) if live[0, w]],
            "xcc_of_dispatch_mod8": {str(r): sorted(set(int(x) for x in blk_xcc[blk_disp % 8 == r])) for r in range(8)},
            "blocks_per_xcc": {str(x): int((blk_xcc == x).sum()) for x in sorted(set(blk_xcc.tolist()))},
            "xcc_by_logical_block": blk_xcc.tolist(),
        }
        # stamps [block][wave][phase]: phase time of a block = its last wave's stamp;
        # waves that do not exist (768-thread blocks: 12 waves) or phases a wave
        # never stamped stay 0 -> NaN
        nw = 16
        v = np.where(v == 0, np.nan, v).reshape(nb, nw, 16)
        t0 = np.nanmin(v[:, :, 0], 1)
        rel = v - t0[:, None, None]
        blk = np.nanmax(rel, 1)             # [nb, phase]: slowest wave of each block
        W = fk.plan.d.W
        reg = fk.plan.reg.reshape(nb, W, W)
        edge = (reg > 0).any(axis=(1, 2))
        corner = (reg < 0).any(axis=(1, 2))
        out["corner_blocks"] = int(corner.sum())
        out["end_by_class"] = {"interior_max": float(blk[~edge, 9].max()) if (~edge).any() else None,
                               "edge_max": float(blk[edge & ~corner, 9].max()) if (edge & ~corner).any() else None,
                               "corner_max": float(blk[corner, 9].max()) if corner.any() else None}
        names = ["start", "window_put", "window_bar"] + sum(
            [[f"s{s}_faces", f"s{s}_upd"] for s in range(1, 4)], []) + ["end"]
        ph = {}
        side = edge & ~corner
        mean = lambda m, k: round(float(blk[m, k].mean()), 0) if m.any() else None
        mean2 = lambda arr, m, k: round(float(arr[m, k].mean()), 0) if m.any() else None
        names = names + [f"s{s}_faces_prebar" for s in range(1, 4)]
        for k, nm in enumerate(names):
            ph[nm] = {"int_mean": mean(~edge, k), "edge_mean": mean(side, k), "corner_mean": mean(corner, k),
                      "max": float(blk[:, k].max())}
        out["phases_cycles"] = ph
        P = fk.plan
        # shader clock from the (memtime, memrealtime) pairs at block start / end
        dt_rt = (v[:, :, 15] - v[:, :, 14]) / 100e6     # seconds (100 MHz)
        dt_sc = (v[:, :, 9] - v[:, :, 0])
        ok = np.isfinite(dt_rt) & np.isfinite(dt_sc) & (dt_rt > 0)
        out["shader_clock_ghz"] = float(np.median(dt_sc[ok] / dt_rt[ok]) / 1e9) if ok.any() else None
        rt0 = np.nanmin(v[:, :, 14])
        out["kernel_span_us_rt"] = float((np.nanmax(v[:, :, 15]) - rt0) / 100.0)
        out["ghost_entries_max"] = int(P.gcnt.max())
        # the same inside a 20-step launch: phases of the last step, from its loop top
        st.zero_()
        md = fk.multi_desc(20)
        md.stamps = st.data_ptr()
        fk.launch(0, nsteps=20)
        torch.cuda.synchronize()
        md.stamps = 0
        fk.check()
        v2 = st.cpu().numpy()[:, :, :16].astype(np.float64).reshape(nb, nw, 16)
        v2 = np.where(v2 == 0, np.nan, v2)
        top = np.nanmin(v2[:, :, 13], 1)
        rel2 = np.nanmax(v2 - top[:, None, None], 1)
        idx = [13, 1, 2, 3, 4, 5, 6, 7, 8, 9]
        nm2 = ["loop_top", "wait_load_put", "bar"] + sum([[f"s{s}_faces", f"s{s}_upd"] for s in range(1, 4)], []) + ["end"]
        # per-wave face-phase time (from the stage's start barrier to the wave's last
        # face task), mean over each block class: which SIMD / wave limits the phase
        starts = {1: 2, 2: 4, 3: 6}
        pw = {}
        for s_ in (1, 2, 3):
            dtw = v2[:, :, 9 + s_] - np.nanmax(v2[:, :, starts[s_]], 1)[:, None]
            with np.errstate(all="ignore"):
                pw[f"s{s_}"] = {c_: [None if np.isnan(x) else int(x) for x in np.nanmean(dtw[m_], 0)]
                                for c_, m_ in (("int", ~edge), ("edge", side), ("corner", corner))}
        out["multi_wave_face_cycles"] = pw
        out["multi_last_step_cycles"] = {n_: {"int": mean2(rel2, ~edge, k), "edge": mean2(rel2, side, k),
                                              "corner": mean2(rel2, corner, k), "max": float(rel2[:, k].max())}
                                         for n_, k in zip(nm2, idx)}
        out["corner_faces_max"] = int(P.ccnt.max())
        out["start_spread"] = float(np.nanmax(t0) - np.nanmin(t0))
        out["end_max"] = float(np.nanmax(np.nanmax(v[:, :, 9], 1) - np.nanmin(t0)))
        out["edge_blocks"] = int(edge.sum())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
