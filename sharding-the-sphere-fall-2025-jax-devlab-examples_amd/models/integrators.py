"""Explicit Runge-Kutta integrators as stage tables.

The reference never names its time integrator; the
framework offers forward Euler, SSP-RK2, SSP-RK3 (default) and classical RK4.
The slide-19 cost model counts work "per rhs eval." (PDF s.19); here every
rhs evaluation is one stage launch.

Every stage is one fused kernel launch (HIP path) computing

    out     = a0 * X + a1 * Q + a2 * dt * L(Q)
    acc_out = c0 * ACC + c1 * X + c2 * dt * L(Q)      (RK4 only)

where Q is the stage input read *with halos* and X / ACC are read only at the
cell being written.  Buffers are named by pool index; ``rotation`` maps the
pool after a step (identity except for Euler, which ping-pongs), so a step is
buffer-invariant after ``period`` steps and can be captured in one hipGraph.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple


@dataclass(frozen=True)
class Stage:
    X: int
    Q: int
    out: int
    a0: float
    a1: float
    a2: float
    acc_in: int = -1
    acc_out: int = -1
    c0: float = 0.0
    c1: float = 0.0
    c2: float = 0.0


@dataclass(frozen=True)
class Integrator:
    name: str
    stages: Tuple[Stage, ...]
    nbuf: int
    rotation: Tuple[int, ...]   # new_pool[i] = old_pool[rotation[i]]
    order: int

    @property
    def period(self) -> int:
        p, perm = 1, list(self.rotation)
        cur = list(perm)
        while cur != list(range(self.nbuf)):
            cur = [perm[c] for c in cur]
            p += 1
        return p


def euler() -> Integrator:
    return Integrator("euler", (Stage(0, 0, 1, 0.0, 1.0, 1.0),), 2, (1, 0), 1)


def ssp_rk2() -> Integrator:
    return Integrator("ssprk2", (
        Stage(0, 0, 1, 0.0, 1.0, 1.0),
        Stage(0, 1, 0, 0.5, 0.5, 0.5),
    ), 2, (0, 1), 2)


def ssp_rk3() -> Integrator:
    return Integrator("ssprk3", (
        Stage(0, 0, 1, 0.0, 1.0, 1.0),
        Stage(0, 1, 2, 0.75, 0.25, 0.25),
        Stage(0, 2, 0, 1.0 / 3.0, 2.0 / 3.0, 2.0 / 3.0),
    ), 3, (0, 1, 2), 3)


def rk4() -> Integrator:
    return Integrator("rk4", (
        Stage(0, 0, 1, 0.0, 1.0, 0.5, acc_in=-1, acc_out=3, c0=0.0, c1=1.0, c2=1.0 / 6.0),
        Stage(0, 1, 2, 1.0, 0.0, 0.5, acc_in=3, acc_out=3, c0=1.0, c1=0.0, c2=1.0 / 3.0),
        Stage(0, 2, 1, 1.0, 0.0, 1.0, acc_in=3, acc_out=3, c0=1.0, c1=0.0, c2=1.0 / 3.0),
        Stage(3, 1, 0, 1.0, 0.0, 1.0 / 6.0),
    ), 4, (0, 1, 2, 3), 4)


INTEGRATORS = {"euler": euler, "ssprk2": ssp_rk2, "ssprk3": ssp_rk3, "rk3": ssp_rk3, "rk4": rk4}


def get_integrator(name: str) -> Integrator:
    try:
        return INTEGRATORS[name.lower()]()
    except KeyError:
        raise ValueError(f"unknown integrator {name!r}; choose from {sorted(INTEGRATORS)}")


def step_kernel_compatible(integ: Integrator) -> bool:
    """True if a whole step can run in one kernel with the state held on
    chip (the fused step, ops/csrc/fused_step.hip): period 1, no accumulator,
    at most 4 stages, every stage combines the step-start state (buffer 0)
    with the previous stage's output (the first stage's input is buffer 0),
    and the last stage writes buffer 0 (SSP-RK2, SSP-RK3)."""
    st = integ.stages
    if integ.period != 1 or not 1 <= len(st) <= 4 or st[-1].out != 0 or st[0].Q != 0:
        return False
    for k, s in enumerate(st):
        if s.X != 0 or s.acc_in >= 0 or s.acc_out >= 0:
            return False
        if k and s.Q != st[k - 1].out:
            return False
    return True
