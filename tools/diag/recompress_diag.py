import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from stsphere.models import tt
from stsphere.ops import tt_ops
orig = tt_ops.recompress
worst = []
lib_err = []
sw_cur = [None]
def wrap(A, B, eps, max_rank=None):
    a, b = orig(A, B, eps, max_rank)
    ref = A @ B.T
    n = float(ref.norm())
    e = float((a @ b.T - ref).norm()) / max(n, 1e-300)
    w = tt.recompress(A, B, eps, max_rank)
    ew = float((w.dense() - ref).norm()) / max(n, 1e-300)
    wl = sw_cur[0]._round_library(A, B)
    el = float((wl.dense() - ref).norm()) / max(n, 1e-300)
    lib_err.append(el)
    # conditioning of the inputs
    sa = torch.linalg.svdvals(A); sb = torch.linalg.svdvals(B)
    worst.append((e, ew, A.shape[0], B.shape[0], A.shape[1], a.shape[1], w.rank,
                  float(sa[-1] / sa[0]), float(sb[-1] / sb[0])))
    return a, b
tt_ops.recompress = wrap
for N in (20, 48):
    worst.clear()
    sw = tt.CubedSphereLowRankShallowWater(N, eps=1e-13, device="cuda", backend="hip")
    sw_cur[0] = sw
    lib_err.clear()
    W = sw.gaussian_hill(); F = sw.to_factored(W)
    F = sw.step(F, sw.dt_max)
    worst.sort(reverse=True)
    print(N, "calls", len(worst))
    for r in worst[:12]:
        print("  err %.2e torch %.2e NA %d NB %d k %d rn %d rt %d condA %.1e condB %.1e" % r)
    print("  host-core library route: max err %.2e" % max(lib_err))
    import collections
    print("  errs>1e-11 by k:", collections.Counter(r[4] for r in worst if r[0] > 1e-11).most_common(10))
