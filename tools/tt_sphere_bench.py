"""Time the six-panel factored linear SWE (models/tt.py::
CubedSphereLowRankShallowWater) against the dense six-panel step of the same
discrete operator on one GPU (verdict r5 item 6; PDF s.3, s.19).

Per N: the "hip" backend (native CholeskyQR3 roundings), optionally the
"torch" backend (rocSOLVER QR + SVD roundings), and ``dense_step``; each
timed over ``--steps`` SSP-RK3 steps after one warm-up step, with the factored
result checked against the dense one.  One JSON line per (N, path) to stdout
and ``--out``.

    python tools/tt_sphere_bench.py --N 256 1024 --eps 1e-10 --steps 2
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stsphere.models import tt  # noqa: E402


def _timed(fn, steps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(steps):
        fn()
        print(f"  step {i + 1}/{steps} {time.perf_counter() - t:.2f}s", flush=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, nargs="+", default=[256, 1024])
    ap.add_argument("--eps", type=float, default=1e-10, help="rounding accuracy (relative)")
    ap.add_argument("--coef-eps", type=float, default=None, help="coefficient factor accuracy (default: --eps)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--torch-backend", action="store_true", help="also time the rocSOLVER QR + SVD roundings")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ce = a.eps if a.coef_eps is None else a.coef_eps
    rows = []

    def emit(r):
        rows.append(r)
        print(json.dumps(r), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(r) + "\n")

    for N in a.N:
        t0 = time.perf_counter()
        sw = tt.CubedSphereLowRankShallowWater(N, eps=a.eps, coef_eps=ce, device="cuda", backend="hip")
        W = sw.gaussian_hill()
        F0 = sw.to_factored(W)
        torch.cuda.synchronize()
        setup = time.perf_counter() - t0
        print(f"N={N}: setup {setup:.1f}s, coefficient ranks {sw.coefficient_ranks()}", flush=True)
        dt = sw.dt_max
        Wd = [W.clone()]
        Wd[0] = sw.dense_step(Wd[0], dt)

        def dstep():
            Wd[0] = sw.dense_step(Wd[0], dt)

        t_dense = _timed(dstep, max(a.steps, 5))
        emit({"N": N, "path": "dense six-panel (torch)", "s_per_step": t_dense, "storage": int(W.numel())})
        backends = ["hip"] + (["torch"] if a.torch_backend else [])
        for be in backends:
            sw.backend = be
            F = [sw.step(F0, dt)]
            sw.stats.update(recompressions=0, native=0, library=0, max_k=0)

            def fstep():
                F[0] = sw.step(F[0], dt)

            t_f = _timed(fstep, a.steps)
            st = dict(sw.stats)
            D = sw.to_dense(F[0])
            Wr = W.clone()
            for _ in range(a.steps + 1):
                Wr = sw.dense_step(Wr, dt)
            err = float((D - Wr).abs().amax() / Wr.abs().amax())
            ranks = [f.rank for Fq in F[0] for f in Fq]
            emit({"N": N, "path": f"factored ({be})", "s_per_step": t_f, "vs_dense": t_f / t_dense,
                  "rel_err_vs_dense": err, "eps": a.eps, "coef_eps": ce, "field_rank_max": max(ranks),
                  "storage": int(sum(f.storage() for Fq in F[0] for f in Fq)),
                  "roundings_per_step": st["recompressions"] / a.steps, "native_calls_per_step": st["native"] / a.steps,
                  "library_per_step": st["library"] / a.steps, "max_k": st["max_k"], "setup_s": setup})
    return rows


if __name__ == "__main__":
    main()
