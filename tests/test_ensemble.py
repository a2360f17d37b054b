"""Ensemble members (ensemble.py): independent runs of one configuration.
CPU: members are the same runs as their engines stepped alone, member 0 is
the unperturbed run, the perturbation gives a non-zero spread.  GPU: the
concurrent native members are bitwise equal to each member run alone."""
import numpy as np
import pytest
import torch

from stsphere.engine import Engine
from stsphere.ensemble import Ensemble
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.parallel.layout import TileLayout


def _alone(grid, L, ens, m, nsteps, device, backend):
    e = Engine(ShallowWater("tc5"), L, grid=grid, device=device, backend=backend, dt=ens.dt)
    e.set_state(ens0_state[m].to(device))
    e.step(nsteps)
    return e.tiles_view().cpu()


ens0_state = {}


def test_ensemble_cpu_members_match_single_runs():
    grid = CubedSphereGrid(8)
    L = TileLayout(8, 1, 1, ng=2)
    ens = Ensemble(lambda: ShallowWater("tc5"), L, 3, amplitude=1e-3, grid=grid)
    for m, e in enumerate(ens.engines):
        ens0_state[m] = e.tiles_view().clone()
    ref = Engine(ShallowWater("tc5"), L, grid=grid, dt=ens.dt)
    assert torch.equal(ens0_state[0], ref.tiles_view())           # member 0 unperturbed
    assert not torch.equal(ens0_state[1], ens0_state[2])
    sp0 = ens.spread()
    assert sp0["spread_rms"] > 0
    ens.run(3)
    for m in range(3):
        assert torch.equal(ens.engines[m].tiles_view(), _alone(grid, L, ens, m, 3, "cpu", "torch"))
    assert ens.states().shape == (3, 4, 6, 8, 8)
    assert ens.global_fields(0).shape == (3, 6, 8, 8)
    with pytest.raises(ValueError):
        Ensemble(lambda: ShallowWater("tc5"), L, 0, grid=grid)


@pytest.mark.gpu
def test_ensemble_native_concurrent_members_bitwise():
    grid = CubedSphereGrid(24)
    L = TileLayout(24, 2, 1, ng=2)
    ens = Ensemble(lambda: ShallowWater("tc5"), L, 2, amplitude=1e-4, grid=grid, device="cuda", backend="hip",
                   steps_per_graph=4)
    assert ens.native
    for m, e in enumerate(ens.engines):
        ens0_state[m] = e.tiles_view().clone()
    ens.prepare(10)
    ens.run(10)                         # chunks 4, 4, 2, interleaved across the members
    torch.cuda.synchronize()
    got = ens.states().cpu()
    for m in range(2):
        alone = _alone(grid, L, ens, m, 10, "cuda", "hip")
        assert torch.equal(got[m], alone), float((got[m] - alone).abs().max())
    ens.close()


def test_ensemble_cli_from_config_cpu():
    import os
    from stsphere.__main__ import run_ensemble
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "sharding-the-sphere-fall-2025-jax-devlab-examples_amd", "configs", "plumbing_cpu.yaml")
    r = run_ensemble(cfg, 2, 1e-3, nsteps=2)
    assert r["members"] == 2 and r["steps"] == 2 and not r["native"]
    assert r["field0_spread_rms_initial"] > 0 and np.isfinite(r["field0_spread_rms_final"])
    r1 = run_ensemble(cfg, 1, 1e-3, nsteps=1)
    assert r1["field0_spread_rms_initial"] == 0.0
