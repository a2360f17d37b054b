"""Williamson et al. (1992) normalised error norms (the survey's test plan,
SURVEY.md section 4: "l1/l2/l-inf error norms versus the analytic/reference
solution; convergence order ~2 for PLR").  The reference itself shows its
advection result only as a picture (PDF s.13 / s.18: "Cosine Bell Advection,
Initial vs Final"); these norms put a number on that comparison.

For a field h and the true solution h_T on the same cells, with I(.) the
area-weighted global integral:

    l1   = I(|h - h_T|) / I(|h_T|)
    l2   = sqrt(I((h - h_T)^2) / I(h_T^2))
    linf = max|h - h_T| / max|h_T|
"""
from __future__ import annotations

import math
from typing import Dict, Sequence

import numpy as np


def williamson_norms(h: np.ndarray, h_true: np.ndarray, area: np.ndarray) -> Dict[str, float]:
    h = np.asarray(h, dtype=np.float64)
    t = np.asarray(h_true, dtype=np.float64)
    a = np.asarray(area, dtype=np.float64)
    if not (h.shape == t.shape == a.shape):
        raise ValueError(f"shape mismatch: {h.shape}, {t.shape}, {a.shape}")
    d = h - t
    return {
        "l1": float((np.abs(d) * a).sum() / (np.abs(t) * a).sum()),
        "l2": float(math.sqrt((d * d * a).sum() / (t * t * a).sum())),
        "linf": float(np.abs(d).max() / np.abs(t).max()),
    }


def convergence_order(errors: Sequence[float], resolutions: Sequence[int]) -> float:
    """Least-squares slope of log(error) against log(1 / N)."""
    x = -np.log(np.asarray(resolutions, dtype=np.float64))
    y = np.log(np.asarray(errors, dtype=np.float64))
    return float(np.polyfit(x, y, 1)[0])
