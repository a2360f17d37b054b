#!/usr/bin/env python
"""Factored diffusion at the slides' operating point (PDF s.19: N = 1024; a
rank-3 field, tools/tt_bench.py's modes): the persistent one-launch step
(ops/csrc/tt_persist.hip) against the round-4 kernel chain and the dense
five-point step (eager launches and replayed from a hipGraph), all per
simulated step, plus the persistent kernel's per-phase shader-clock stamps.
One JSON line.

    python tools/tt_persist_probe.py [--N 1024] [--substeps 2]
"""
import argparse
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--substeps", type=int, default=2)
    ap.add_argument("--eps", type=float, default=1e-8)
    a = ap.parse_args()
    import torch
    from stsphere.models import tt
    from stsphere.ops import tt_ops
    N = a.N
    dev = torch.device("cuda")
    x = torch.linspace(0, 1, N + 2, dtype=torch.float64, device=dev)[1:-1]
    A = torch.stack([torch.sin(math.pi * x), 0.3 * torch.sin(3 * math.pi * x), 0.1 * torch.sin(5 * math.pi * x)], 1)
    B = torch.stack([torch.sin(2 * math.pi * x), torch.sin(math.pi * x), torch.sin(4 * math.pi * x)], 1)
    A, B = A.contiguous(), B.contiguous()
    s = tt.LowRankDiffusion(N, kappa=1.0, eps=a.eps, backend="hip", device=dev, substeps=a.substeps)
    dt = 0.5 * s.dt_max
    c = dt / (s.h * s.h)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    out = {"N": N, "rank": 3, "substeps": a.substeps, "eps": a.eps}

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    # dense five-point step, eager and graph-replayed
    U = (A @ B.T).contiguous()
    V = torch.empty_like(U)
    st = {"u": U, "v": V}

    def dense():
        tt_ops.dense_diffusion(st["u"], c, out=st["v"])
        st["u"], st["v"] = st["v"], st["u"]
    out["dense_eager_us_per_step"] = timed(dense, 200)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            dense()
    torch.cuda.current_stream().wait_stream(side)
    with torch.cuda.graph(g):
        for _ in range(20):
            dense()
    out["dense_graph_us_per_step"] = timed(g.replay, 20) / 20
    # round-4 chain: one native call per factored step
    lr = {"f": tt.LowRankField(A.clone(), B.clone())}

    def chain():
        lr["f"] = s.step(lr["f"], dt)
    out["chain_us_per_step"] = timed(chain, 20) / a.substeps
    # persistent: ncalls factored steps per launch
    for nc in (1, 10, 50):
        f0 = tt.LowRankField(A.clone(), B.clone())
        res = {}

        def pers():
            res["f"] = s.run_persistent(f0, dt, nc)
        out[f"persist_{nc}_us_per_step"] = timed(pers, 10) / (nc * a.substeps)
        out[f"persist_{nc}_rank"] = res["f"].rank
    # accuracy after 50 calls against dense stepping
    f = s.run_persistent(tt.LowRankField(A.clone(), B.clone()), dt, 50)
    sd = tt.LowRankDiffusion(N, kappa=1.0, device=dev)
    Ud = A @ B.T
    for _ in range(50 * a.substeps):
        Ud = sd.dense_step(Ud, dt)
    out["persist_rel_diff_vs_dense"] = float((f.dense() - Ud).norm() / Ud.norm())
    # per-phase stamps of a 10-step launch (shader clocks; wg 0 = A, wg 1 = B)
    nc = 10
    stamps = torch.zeros((nc, 2, 16), dtype=torch.int64, device=dev)
    s.run_persistent(tt.LowRankField(A.clone(), B.clone()), dt, nc, stamps=stamps)
    v = stamps.cpu().numpy().astype(float)
    names = ["start", "expanded", "qr1", "qr2", "qr3", "core_in", "core_out", "product"]
    ph = {}
    for side_, lab in ((0, "A"), (1, "B")):
        d = {}
        for k in range(1, 8):
            d[f"{names[k - 1]}->{names[k]}"] = float(((v[2:, side_, k] - v[2:, side_, k - 1])).mean())
        d["step"] = float(((v[3:, side_, 0] - v[2:-1, side_, 0])).mean())
        # inside CholeskyQR pass 1: Gram partials, Gram reduce, Cholesky + R^-1, row update
        for lab2, (k0, k1) in (("qr1_gram", (1, 8)), ("qr1_reduce", (8, 9)), ("qr1_chol", (9, 10)),
                               ("qr1_update", (10, 2))):
            d[lab2] = float(((v[2:, side_, k1] - v[2:, side_, k0])).mean())
        ph[lab] = d
    out["persist_phase_cycles"] = ph
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
