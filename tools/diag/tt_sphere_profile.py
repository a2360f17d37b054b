"""Where a six-panel factored SWE step (backend "hip") spends its time: host
profile of one step at N (cProfile, top functions) and the wall time of the
native rounding calls alone.  Run under rocprofv3 --kernel-trace --stats for
the device side."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from stsphere.models import tt  # noqa: E402
from stsphere.ops import tt_ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sw = tt.CubedSphereLowRankShallowWater(N, eps=1e-10, coef_eps=1e-10, device="cuda", backend="hip")
W = sw.gaussian_hill()
F = sw.to_factored(W)
F = sw.step(F, sw.dt_max)
torch.cuda.synchronize()
orig = tt_ops.recompress
acc = {"t": 0.0, "n": 0, "k": 0}


def timed(*a, **kw):
    t = time.perf_counter()
    out = orig(*a, **kw)
    acc["t"] += time.perf_counter() - t
    acc["n"] += 1
    acc["k"] += a[0].shape[1]
    return out


tt_ops.recompress = timed
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
F = sw.step(F, sw.dt_max)
torch.cuda.synchronize()
pr.disable()
dt = time.perf_counter() - t0
print(f"N={N}: step {dt:.3f} s; native calls {acc['n']} taking {acc['t']:.3f} s "
      f"({1e6 * acc['t'] / max(1, acc['n']):.0f} us each, mean k {acc['k'] / max(1, acc['n']):.1f})", flush=True)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
