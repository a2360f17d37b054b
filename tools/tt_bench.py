#!/usr/bin/env python
"""Factored (d = 2 TT) diffusion vs the dense five-point step on one MI355X.

The reference models the TT route on its slide 19 (PDF s.19: at N = 1024 and
r = 10 a ~144x total saving over FV-PLR, arithmetic intensity 17.5 vs 0.25);
this measures it.  Per N:

* dense: one N x N explicit step U + c lap(U) (ops/tt_ops.dense_diffusion,
  memory-bound: 16 B per cell at best);
* tt:    one step of models/tt.LowRankDiffusion(backend="hip") on U = A B^T
  (rank-2r expansion, MFMA Gram matrices, host 2r x 2r eigen/SVD, MFMA
  tall-skinny products), wall time per step including the host round trip.

The initial field is an analytic sum of separable modes (rank 3, nothing
decomposed), so N can go to 32768 (8.6 GB per dense fp64 field).  Where the
dense field fits comfortably, the two answers are compared after the timed
steps.  A second table times the MFMA kernels alone on tall operands.

    python tools/tt_bench.py [--sizes 1024,4096,16384,32768] [--steps 20] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def modes(N, device):
    import torch
    x = torch.linspace(0, 1, N + 2, dtype=torch.float64, device=device)[1:-1]
    A = torch.stack([torch.sin(math.pi * x), 0.3 * torch.sin(3 * math.pi * x), 0.1 * torch.sin(5 * math.pi * x)], 1)
    B = torch.stack([torch.sin(2 * math.pi * x), torch.sin(math.pi * x), torch.sin(4 * math.pi * x)], 1)
    return A.contiguous(), B.contiguous()


def time_loop(fn, steps, sync):
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,4096,16384,32768")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--eps", type=float, default=1e-8)
    ap.add_argument("--max-rank", type=int, default=16)
    ap.add_argument("--json", default=None)
    ap.add_argument("--qr", default="cholqr3n", choices=["cholqr3", "cholqr3n", "gram"],
                    help="hip recompression: device CholeskyQR3 (default) or the native Gram/eigen step")
    ap.add_argument("--core", default="device", choices=["device", "host"],
                    help="cholqr3n: the k x k core (Jacobi SVD) on the device (k <= 32) or on the host")
    ap.add_argument("--substeps", default="1,2,3",
                    help="explicit steps per recompression (tt us is per simulated step)")
    a = ap.parse_args()
    import torch
    from stsphere.models import tt
    from stsphere.ops import tt_ops
    dev = torch.device("cuda")
    sync = torch.cuda.synchronize
    rows = []
    print(f"{'N':>6} {'subs':>4} {'rank':>4} {'dense us':>10} {'dense GB/s':>10} {'tt us':>8} {'speedup':>8} "
          f"{'rel diff':>9}")
    def rel_diff_chunked(lr, U):
        """||A B^T - U|| / ||U|| over row blocks (no second N x N matrix)."""
        num = den = 0.0
        for i0 in range(0, U.shape[0], 2048):
            R = lr.A[i0:i0 + 2048] @ lr.B.T
            num += float(((R - U[i0:i0 + 2048]) ** 2).sum())
            den += float((U[i0:i0 + 2048] ** 2).sum())
        return (num / den) ** 0.5

    subs = [int(v) for v in a.substeps.split(",")]
    for N in [int(s) for s in a.sizes.split(",")]:
        A, B = modes(N, dev)
        s0 = tt.LowRankDiffusion(N, kappa=1.0, eps=a.eps, max_rank=a.max_rank, backend="hip", device=dev)
        dt = 0.5 * s0.dt_max
        c = dt * s0.kappa / (s0.h * s0.h)
        U = A @ B.T
        V = torch.empty_like(U)
        state = {"u": U, "v": V}

        def dense_step():
            tt_ops.dense_diffusion(state["u"], c, out=state["v"])
            state["u"], state["v"] = state["v"], state["u"]
        dense_step()
        t_dense = time_loop(dense_step, a.steps, sync)
        for ns in subs:
            s = tt.LowRankDiffusion(N, kappa=1.0, eps=a.eps, max_rank=min(a.max_rank, 64 >> ns), backend="hip", device=dev,
                                    substeps=ns, qr=a.qr, core=a.core)
            st = {"lr": tt.LowRankField(A.clone(), B.clone())}

            def tt_step():
                st["lr"] = s.step(st["lr"], dt)
            for _ in range(2):
                tt_step()
            # same simulated time on both sides before the comparison
            st["lr"] = tt.LowRankField(A.clone(), B.clone())
            state["u"], state["v"] = A @ B.T, torch.empty_like(U)
            calls = max(1, a.steps // ns)
            t_tt = time_loop(tt_step, calls, sync) / ns          # per simulated step
            for _ in range(calls * ns):
                dense_step()
            sync()
            diff = rel_diff_chunked(st["lr"], state["u"])
            row = {"N": N, "qr": a.qr, "substeps": ns, "rank": st["lr"].rank, "dense_us": 1e6 * t_dense,
                   "dense_GBps": 16.0 * N * N / t_dense / 1e9, "tt_us": 1e6 * t_tt, "speedup": t_dense / t_tt,
                   "rel_diff": diff, "steps": calls * ns}
            rows.append(row)
            print(f"{N:>6} {ns:>4} {row['rank']:>4} {row['dense_us']:>10.1f} {row['dense_GBps']:>10.0f} "
                  f"{row['tt_us']:>8.1f} {row['speedup']:>8.2f} {diff:>9.2e}", flush=True)
            del st
        del U, V, state
        torch.cuda.empty_cache()

    # MFMA kernels alone on tall operands (events around 20 back-to-back calls)
    krows = []
    print(f"\n{'kernel':>6} {'rows':>9} {'k':>3} {'m':>3} {'us':>9} {'GB/s':>7} {'TFLOP/s':>8}")
    for N, k, m in [(1 << 22, 32, 32), (1 << 22, 48, 48), (1 << 22, 64, 64), (1 << 24, 32, 16)]:
        X = torch.randn(N, k, dtype=torch.float64, device=dev)
        Y = torch.randn(k, m, dtype=torch.float64, device=dev)
        O = torch.empty(N, m, dtype=torch.float64, device=dev)
        G = torch.empty(k, k, dtype=torch.float64, device=dev)
        work = torch.empty(tt_ops.gram_blocks(N) * 64 * 64, dtype=torch.float64, device=dev)
        for name, fn, nbytes, flops in (
                ("gram", lambda: tt_ops.gram(X, X, out=G, work=work), 8.0 * N * k, 2.0 * N * k * k),
                ("tsmm", lambda: tt_ops.tsmm(X, Y, out=O), 8.0 * N * (k + m), 2.0 * N * k * m)):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            sync()
            us = 1e3 * e0.elapsed_time(e1) / 20
            r = {"kernel": name, "rows": N, "k": k, "m": m if name == "tsmm" else k, "us": us,
                 "GBps": nbytes / us / 1e3, "TFLOPs": flops / us / 1e6}
            krows.append(r)
            print(f"{name:>6} {N:>9} {k:>3} {r['m']:>3} {us:>9.1f} {r['GBps']:>7.0f} {r['TFLOPs']:>8.2f}", flush=True)
        del X, Y, O, G, work
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"diffusion": rows, "kernels": krows, "device": torch.cuda.get_device_name()}, f, indent=1)


if __name__ == "__main__":
    main()
