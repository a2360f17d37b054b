"""Memory-corruption screen: after a trigger sequence (``--trigger``: the
loopback fused kernel, the plain fused kernel, or none), build torch-backend
engines repeatedly and check that their tables do not change while they step
and that every state stays finite.  Prints one line per round and a summary.

    python tools/diag_alias.py --trigger loopback --rounds 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from stsphere.engine import Engine  # noqa: E402
from stsphere.models.geometry import CubedSphereGrid  # noqa: E402
from stsphere.models.swe import ShallowWater  # noqa: E402
from stsphere.parallel.layout import TileLayout  # noqa: E402


def trigger(kind, N=32, t=2):
    from stsphere.ops.fused import FusedKernel
    grid = CubedSphereGrid(N)
    L = TileLayout(N, t, 1, ng=2)
    a = Engine(ShallowWater("tc5"), L, grid=grid, dtype=torch.float64, device="cuda", backend="hip")
    fa = FusedKernel(a)
    fa.step(3)
    fa.launch(0, nsteps=4)
    if kind == "loopback":
        Llb = TileLayout(N, t, 1, ng=2, loopback=True)
        b = Engine(ShallowWater("tc5"), Llb, grid=grid, dtype=torch.float64, device="cuda", backend="hip", dt=a.dt)
        fb = FusedKernel(b, B=fa.plan.B)
        fb.step(3)
        fb.launch(0, nsteps=4)
        torch.cuda.synchronize()
        fb.check()
        ok = torch.equal(a.tiles_view(), b.tiles_view())
        fb.close()
        print("loopback equal", ok, flush=True)
    torch.cuda.synchronize()


def screen(rounds):
    bad = 0
    for r in range(rounds):
        N, t = 24, 1 + (r % 2)
        grid = CubedSphereGrid(N)
        L = TileLayout(N, t, 1, ng=2)
        e = Engine(ShallowWater("tc6", limiter=3), L, grid=grid, dtype=torch.float64, device="cuda",
                   backend="torch")
        torch.cuda.synchronize()
        snap = {k: v.clone() for k, v in e.tens.items() if torch.is_tensor(v)}
        msgs = []
        for k in range(4):
            e.step(1)
            torch.cuda.synchronize()
            nf = int((~torch.isfinite(e.tiles_view())).sum())
            ch = [n for n, v in snap.items() if not torch.equal(v, e.tens[n])]
            if nf or ch:
                msgs.append(f"step {k + 1}: non-finite {nf} changed {ch}")
        bad += bool(msgs)
        print(f"round {r} t={t}: " + ("; ".join(msgs) if msgs else "clean"), flush=True)
    print(f"SUMMARY corrupted rounds {bad} of {rounds}", flush=True)
    return bad


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--trigger", choices=["loopback", "plain", "none"], default="loopback")
    p.add_argument("--rounds", type=int, default=20)
    p.add_argument("--repeat", type=int, default=1, help="trigger + screen cycles")
    a = p.parse_args()
    tot = 0
    for _ in range(a.repeat):
        if a.trigger != "none":
            trigger(a.trigger)
        tot += screen(a.rounds)
    sys.exit(1 if tot else 0)
