#!/usr/bin/env python
"""Where a multi-step fused launch's fixed cost sits (C96, B = 16).

tools/ramp_probe.py fits the GPU-event time of one launch of n steps as
T(n) ~ 10.7 n + 13 us.  This probe separates that constant into the part
inside the kernel and the part outside it.  For n in --ns it launches the
n-step kernel with phase stamps on and reads, per block, the constant-rate
clock (100 MHz) at block start (slot 14) and block end (slot 15):

- dispatch spread: last block start - first block start;
- kernel span: last block end - first block start;
- event time of the same launch (hipEvents around it).

A linear fit of the span over n gives the in-kernel per-step cost and the
in-kernel constant; event - span is the launch overhead outside the kernel.
One JSON line.

    python tools/diag/ramp_stamps.py [--ns 2,4,8,20,60] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="2,4,8,20,60")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from stsphere.engine import Engine
    from stsphere.models.geometry import CubedSphereGrid
    from stsphere.models.swe import ShallowWater
    from stsphere.ops.fused import FusedKernel
    from stsphere.parallel.layout import TileLayout
    L = TileLayout(96, 2, 1, ng=2)
    e = Engine(ShallowWater("tc5"), L, grid=CubedSphereGrid(96), device="cuda", backend="hip")
    fk = FusedKernel(e)
    nb = fk.plan.nb
    FW = 32
    st = torch.zeros((nb, 16, FW), dtype=torch.int64, device="cuda")
    ns = [int(x) for x in a.ns.split(",")]
    out = {"blocks": nb, "B": fk.plan.B, "handoff": getattr(fk, "handoff", None), "rows": {}}
    for n in ns + [1]:
        fk.launch(0, nsteps=n) if n > 1 else fk.launch(0)      # warm
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for n in [1] + ns:
        spans, spreads, evs, ends = [], [], [], []
        for _ in range(a.reps):
            st.zero_()
            if n > 1:
                md = fk.multi_desc(n)
                md.stamps = st.data_ptr()
            else:
                for d in fk.descs:
                    d.stamps = st.data_ptr()
            torch.cuda.synchronize()
            ev0.record()
            fk.launch(0, nsteps=n) if n > 1 else fk.launch(0)
            ev1.record()
            torch.cuda.synchronize()
            if n > 1:
                md.stamps = 0
            else:
                for d in fk.descs:
                    d.stamps = 0
            v = st.cpu().numpy()[:, :, :16].astype(np.float64)
            s0 = np.where(v[:, :, 14] == 0, np.nan, v[:, :, 14])
            s1 = np.where(v[:, :, 15] == 0, np.nan, v[:, :, 15])
            bstart = np.nanmin(s0, 1)
            bend = np.nanmax(s1, 1)
            t0 = np.nanmin(bstart)
            spans.append(float((np.nanmax(bend) - t0) / 100.0))
            spreads.append(float((np.nanmax(bstart) - t0) / 100.0))
            ends.append(float((np.nanmax(bend) - np.nanmin(bend)) / 100.0))
            evs.append(ev0.elapsed_time(ev1) * 1e3)
        fk.check()
        out["rows"][str(n)] = {"event_us": round(statistics.median(evs), 2),
                               "span_us": round(statistics.median(spans), 2),
                               "start_spread_us": round(statistics.median(spreads), 2),
                               "end_spread_us": round(statistics.median(ends), 2)}
    xs = np.array([n for n in ns], dtype=float)
    sp = np.array([out["rows"][str(n)]["span_us"] for n in ns])
    evv = np.array([out["rows"][str(n)]["event_us"] for n in ns])
    b, c = np.polyfit(xs, sp, 1)
    be, ce = np.polyfit(xs, evv, 1)
    out["fit_span"] = {"per_step_us": round(float(b), 3), "const_us": round(float(c), 2)}
    out["fit_event"] = {"per_step_us": round(float(be), 3), "const_us": round(float(ce), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
