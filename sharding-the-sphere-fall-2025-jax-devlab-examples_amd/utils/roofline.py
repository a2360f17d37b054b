"""Roofline and Tensor-Train cost model (PDF s.5, s.19).

Reproduces the slide-19 analytic model and evaluates it for MI355X:

* roofline: attainable = min(peak_flops, AI * peak_bw); ridge = peak / bw
  (slide example "TPU v4 class": 900 GB/s, 275 TFLOP/s, ridge 305.6)
* FV-PLR: 870 flops / cell at AI ~0.25 flop/byte (unfused XLA traffic)
* TT-FV (slide 3 / 19): N x N fields compressed to O(d N r^2); per
  "100 flops/var/cell/rhs eval." the dense cost is 100 N^2, the TT cost is
  dominated by r x r x r contractions.

The TT part is the slide's analytic model with its constants back-solved from
the plotted curves (see ``TT_*`` below); it is a model, not a measurement.
``models/tt.py`` implements actual TT numerics.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List


@dataclass(frozen=True)
class Machine:
    name: str
    peak_flops: float     # FLOP/s
    peak_bw: float        # B/s

    @property
    def ridge(self) -> float:
        return self.peak_flops / self.peak_bw

    def attainable(self, ai: float) -> float:
        return min(self.peak_flops, ai * self.peak_bw)


TPU_V4_CLASS = Machine("TPU v4 class (slide 19)", 275e12, 900e9)
MI355X_FP64 = Machine("MI355X fp64 vector", 78.6e12, 8.0e12)
MI355X_FP32 = Machine("MI355X fp32 vector", 157.3e12, 8.0e12)
MI355X_FP64_MEASURED_BW = Machine("MI355X fp64, measured stream BW", 78.6e12, 6.29e12)

FV_PLR_FLOPS_PER_CELL = 870.0
FV_PLR_AI = 0.25


def fv_plr_cell_rate(m: Machine, flops_per_cell: float = FV_PLR_FLOPS_PER_CELL, ai: float = FV_PLR_AI) -> float:
    """Cell updates per second on the roofline."""
    return m.attainable(ai) / flops_per_cell


def fused_ai(flops_per_cell: float, bytes_per_cell: float) -> float:
    return flops_per_cell / bytes_per_cell


# Slide-19 TT model, back-solved from the slide's own curves (N = 1024,
# "100 flops/var/cell/rhs eval."): TT flops ~ 12.3 N r^3 (the r^3 factor is the
# "r x r x r multiplies"), TT storage ~ 2 N r^2 words (the O(d N r^2) of slide 3
# with d = 2), TT arithmetic intensity ~ 1.75 r flop/byte, and the plotted
# "total savings" = flop reduction x TT arithmetic intensity.  These constants
# reproduce every value read off the chart (8.3x/5.3x/AI 17.5/~144x at r = 10,
# 2.0x/2.0x/28/56x at r = 16, ...) within the +-10 % reading error.
TT_FLOP_COEF = 12.3
TT_MEM_WORDS_COEF = 2.0
TT_AI_PER_RANK = 1.75


def tt_costs(N: int = 1024, r: int = 10, flops_per_var_cell: float = 100.0) -> Dict[str, float]:
    dense_flops = flops_per_var_cell * N * N
    dense_words = float(N * N)
    tt_flops = TT_FLOP_COEF * N * r ** 3
    tt_words = TT_MEM_WORDS_COEF * N * r ** 2
    tt_ai = TT_AI_PER_RANK * r
    flop_red = dense_flops / tt_flops
    return {"N": N, "r": r, "dense_flops": dense_flops, "tt_flops": tt_flops, "flop_reduction": flop_red,
            "dense_words": dense_words, "tt_words": tt_words, "memory_reduction": dense_words / tt_words,
            "tt_ai": tt_ai, "total_savings": flop_red * tt_ai}


def tt_savings_table(N: int = 1024, ranks: List[int] = (10, 12, 14, 16, 18, 20, 25, 30)) -> List[Dict[str, float]]:
    return [tt_costs(N, r) for r in ranks]


def tt_time_on(m: Machine, N: int, r: int, dense_ai: float = FV_PLR_AI) -> Dict[str, float]:
    """Roofline times (s) of one RHS evaluation, dense FV vs TT, on machine m."""
    c = tt_costs(N, r)
    td = c["dense_flops"] / m.attainable(dense_ai)
    tt = c["tt_flops"] / m.attainable(c["tt_ai"])
    return {"dense_s": td, "tt_s": tt, "speedup": td / tt}


def report() -> str:
    lines = ["Roofline model (PDF s.19)"]
    for m in (TPU_V4_CLASS, MI355X_FP64, MI355X_FP32):
        lines.append(f"  {m.name:32s} ridge {m.ridge:7.1f} flop/B; FV-PLR @AI 0.25: "
                     f"{m.attainable(FV_PLR_AI) / 1e9:8.1f} GF/s = {fv_plr_cell_rate(m):.3e} cell-updates/s")
    lines.append("TT vs dense (N = 1024, 100 flops/var/cell/rhs), slide-19 model:")
    for c in tt_savings_table():
        mi = tt_time_on(MI355X_FP64, 1024, c["r"])
        lines.append(f"  r={c['r']:3d}: flops x{c['flop_reduction']:.2f}  memory x{c['memory_reduction']:.2f}  "
                     f"AI {c['tt_ai']:.1f}  total x{c['total_savings']:.0f}   (MI355X fp64 roofline speedup "
                     f"x{mi['speedup']:.0f})")
    return "\n".join(lines)


if __name__ == "__main__":
    print(report())
