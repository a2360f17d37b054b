"""Driver, config, checkpoint/restart, history, metrics, zarr."""
import os

import numpy as np
import pytest
import yaml

import stsphere as S
from stsphere.utils import checkpoint as ckpt, zarr_lite
from stsphere.utils.history import read_history, read_metrics


def _cfg(tmp, nd=1, t=1, **io):
    return {"parallelization": {"tiles_per_edge": t, "num_devices": nd, "device_type": "cpu"},
            "grid": {"N": 8}, "physics": {"model": "swe", "case": "tc2"}, "time": {"nsteps": 4},
            "io": dict({"output_dir": str(tmp)}, **io)}


def test_config_roundtrip_and_errors(tmp_path):
    c = S.load_config(_cfg(tmp_path))
    p = tmp_path / "c.yaml"
    S.save_config(c, str(p))
    assert S.load_config(str(p)).to_dict() == c.to_dict()
    with pytest.raises(ValueError):
        S.load_config({"parallelization": {"bogus": 1}})
    assert S.load_config("parallelization:\n  num_devices: 2\n").parallelization.num_devices == 2


def test_shipped_configs_parse():
    here = os.path.join(S.__path__[0], "configs")
    files = [f for f in os.listdir(here) if f.endswith(".yaml")]
    assert files
    for f in files:
        S.load_config(os.path.join(here, f))


def test_checkpoint_partition_independent(tmp_path):
    s = S.Solver(_cfg(tmp_path, nd=8, t=2, checkpoint_interval=2), verbose=False)
    s.run()
    assert ckpt.list_checkpoints(os.path.join(str(tmp_path), "checkpoints")) == [2, 4]
    ref = s.gather_global()
    # any tiling reads it back exactly
    s1 = S.Solver(_cfg(tmp_path, nd=3, t=1, restore="latest"), verbose=False)
    s1.initialize()
    assert s1.step_count == 4 and np.array_equal(s1.gather_global(), ref)
    # continuing on another rank count or another tiling equals continuing the
    # original (panel-edge pairs are chosen on the whole edge),
    # and a t = 2 checkpoint resumed at t = 1 equals a t = 1 run from the start
    s2 = S.Solver(_cfg(tmp_path, nd=3, t=2, restore="latest"), verbose=False)
    s2.initialize()
    s.step(2)
    s2.step(2)
    s1.step(2)
    assert np.array_equal(s2.gather_global(), s.gather_global())
    a, b = s1.gather_global(), s.gather_global()
    assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max()
    s0 = S.Solver(_cfg(tmp_path / "fresh", nd=1, t=1), verbose=False)
    s0.run(nsteps=6)
    c = s0.gather_global()
    assert np.abs(a - c).max() <= 1e-12 * np.abs(c).max()


def test_incomplete_checkpoint_ignored(tmp_path):
    s = S.Solver(_cfg(tmp_path, checkpoint_interval=2), verbose=False)
    s.run()
    d = ckpt.latest_checkpoint(str(tmp_path / "checkpoints"))
    os.remove(os.path.join(d, ckpt.COMMIT))
    assert ckpt.latest_checkpoint(str(tmp_path / "checkpoints")).endswith("00000002")


def test_history_and_metrics(tmp_path):
    s = S.Solver(_cfg(tmp_path, nd=2, history_interval=2, metrics_interval=1), verbose=False)
    s.run()
    h = read_history(str(tmp_path / "history.zarr"), "h")
    assert h.shape == (3, 6, 8, 8) and np.allclose(h[-1], s.global_field("h"))
    t = zarr_lite.read_array(str(tmp_path / "history.zarr"), "time")
    assert np.allclose(t, [0, 2 * s.dt, 4 * s.dt])
    m = read_metrics(str(tmp_path / "metrics.jsonl"))
    assert len(m) == 4 and "mass" in m[-1] and m[-1]["step"] == 4


def test_watchdog_raises_on_nan(tmp_path):
    c = _cfg(tmp_path)
    c["runtime"] = {"watchdog_interval": 1}
    c["time"]["dt"] = 1e6          # violently unstable
    c["time"]["nsteps"] = 50
    s = S.Solver(c, verbose=False)
    with pytest.raises(FloatingPointError):
        s.run()


def test_watchdog_recovers_from_checkpoint(tmp_path):
    c = _cfg(tmp_path, checkpoint_interval=2)
    c["runtime"] = {"watchdog_interval": 1}
    s = S.Solver(c, verbose=False)
    s.initialize()
    dt0 = s.dt
    s.run(nsteps=2)                # good checkpoint at step 2
    s.cfg.io.checkpoint_interval = 0
    s.set_dt(dt0 * 8)              # unstable from here on
    t1 = s.time
    out = s.run(nsteps=40)         # watchdog: restore step 2, halve the current dt, until stable
    assert s.all_finite() and out["recoveries"] >= 1
    # each recovery halves the dt in use (not the checkpoint's), and the run
    # still ends at the requested simulated time
    assert s.dt == dt0 * 8 / 2 ** out["recoveries"]
    assert abs(s.time - (t1 + 40 * 8 * dt0)) < 1e-6 * s.time
    assert out["steps_run"] > 40


def test_checkpoints_between_watchdog_intervals_hold_finite_states(tmp_path):
    """Checkpoint interval 2, watchdog interval 3 (not aligned): a checkpoint
    that falls between watchdog checks tests the state first, so no saved
    checkpoint ever holds a non-finite state and recovery always finds a good
    one."""
    c = _cfg(tmp_path, checkpoint_interval=2, keep_checkpoints=3)
    c["runtime"] = {"watchdog_interval": 3}
    s = S.Solver(c, verbose=False)
    s.initialize()
    s.set_dt(s.dt * 64)            # blows up within a few steps
    try:
        s.run(nsteps=30)
    except FloatingPointError:
        pass
    root = os.path.join(str(tmp_path), "checkpoints")
    steps = ckpt.list_checkpoints(root)
    assert steps
    for st in steps:
        vals = ckpt.read_fields(ckpt.step_dir(root, st))
        assert all(np.isfinite(v).all() for v in vals.values()), st


def test_history_frames_follow_simulated_time_across_recovery(tmp_path):
    """After a watchdog rollback the replayed interval overwrites its own
    history frames (frames are indexed by simulated time, not by a counter)."""
    c = _cfg(tmp_path, checkpoint_interval=2, history_interval=2)
    c["runtime"] = {"watchdog_interval": 1}
    s = S.Solver(c, verbose=False)
    s.initialize()
    dt0 = s.dt
    s.set_dt(dt0 * 8)
    out = s.run(nsteps=6)
    t = zarr_lite.read_array(str(tmp_path / "history.zarr"), "time")
    assert out["recoveries"] >= 1 and len(t) == 4
    assert np.allclose(t, [0, 16 * dt0, 32 * dt0, 48 * dt0])
    h = read_history(str(tmp_path / "history.zarr"), "h")
    assert np.isfinite(h).all() and np.allclose(h[-1], s.global_field("h"))


def test_run_chunks_follow_io_intervals(tmp_path):
    """Chunk lengths come from the I/O intervals, so every interval boundary
    is hit exactly (metrics at 3, 6, 9, history at 0, 4, 8, 10 = end)."""
    s = S.Solver(_cfg(tmp_path, history_interval=4, metrics_interval=3), verbose=False)
    out = s.run(nsteps=10)
    m = read_metrics(str(tmp_path / "metrics.jsonl"))
    assert [r["step"] for r in m] == [3, 6, 9, 10]
    t = zarr_lite.read_array(str(tmp_path / "history.zarr"), "time")
    assert np.allclose(t, [0, 4 * s.dt, 8 * s.dt])
    assert out["steps_run"] == 10 and set(out["phase_s"]) >= {"step", "history", "metrics"}


def test_run_summary_reports_williamson_norms(tmp_path):
    """TC2 has a closed-form solution (steady state): the run summary carries
    its l1 / l2 / linf errors; TC5 has none and reports no norms."""
    s = S.Solver(S.load_config(_cfg(tmp_path)), verbose=False)
    out = s.run(nsteps=4)
    assert 0 < out["err_l2"] < 1e-2 and 0 < out["err_linf"] < 1e-2 and out["err_l1"] > 0
    c = _cfg(tmp_path)
    c["physics"]["case"] = "tc5"
    s5 = S.Solver(S.load_config(c), verbose=False)
    assert "err_l2" not in s5.run(nsteps=2) and s5.error_norms() is None


def test_geometry_and_initial_condition_zarr_stages(tmp_path):
    """Pipeline stages of PDF s.6: the first run writes the grid and the
    initial condition as zarr groups; a second run (another partition) reads
    them and reproduces the first run bitwise."""
    io = {"geometry": str(tmp_path / "grid.zarr"), "initial_condition": str(tmp_path / "ic.zarr")}
    s = S.Solver(_cfg(tmp_path / "a", nd=1, **io), verbose=False)
    s.initialize()
    assert zarr_lite.read_attrs(io["geometry"])["N"] == 8
    assert set(zarr_lite.list_arrays(io["initial_condition"])) == set(s.fields)
    ic = s.gather_global()
    s.run(nsteps=3)
    # second run: geometry and IC come from the zarr groups
    from stsphere.models.geometry import CubedSphereGrid
    s2 = S.Solver(_cfg(tmp_path / "b", nd=6, **io), verbose=False)
    s2.initialize()
    assert np.array_equal(s2.gather_global(), ic)
    assert np.array_equal(s2.grid.x_edge_normals(), CubedSphereGrid(8).x_edge_normals())
    s2.run(nsteps=3)
    assert np.array_equal(s2.gather_global(), s.gather_global())
    # a changed IC on disk is what the next run starts from
    zarr_lite.write_array(io["initial_condition"], "h", ic[0] * 1.01, chunks=(1, 8, 8))
    s3 = S.Solver(_cfg(tmp_path / "c", nd=1, **io), verbose=False)
    s3.initialize()
    assert np.array_equal(s3.gather_global()[0], ic[0] * 1.01)
    with pytest.raises(ValueError):
        S.Solver(dict(_cfg(tmp_path / "d", **io), grid={"N": 12}), verbose=False).initialize()
    # same fields and grid, another SWE case (TC5 has topography): refused
    with pytest.raises(ValueError, match="case"):
        S.Solver(dict(_cfg(tmp_path / "e", **io), physics={"model": "swe", "case": "tc5"}),
                 verbose=False).initialize()


def test_plot_cli_products(tmp_path):
    """`stsphere plot` renders the s.12 sphere frames, the s.13 equatorial
    band and the s.18 six-panel from a run's history."""
    from stsphere.__main__ import main
    s = S.Solver(_cfg(tmp_path, history_interval=2), verbose=False)
    s.run()
    out = tmp_path / "plots"
    assert main(["plot", str(tmp_path / "history.zarr"), "h", str(out)]) == 0
    names = {p.name for p in out.rglob("*.png")}
    assert {"h_band_initial.png", "h_band_final.png", "h_six_panel.png", "h_0000.png"} <= names


def test_host_queue_threaded_keeps_order_and_raises():
    """Solver.run's background writer (_HostQueue): items run in submission
    order, drain(block=True) waits for all, a failing item raises at the next
    drain, clear() drops what has not started."""
    import threading
    import time
    from stsphere.driver import _HostQueue
    q = _HostQueue(threaded=True)
    out = []
    gate = threading.Event()
    q.append((None, lambda: (gate.wait(5), out.append(1))))
    for k in range(2, 6):
        q.append((None, lambda k=k: out.append(k)))
    q.drain()                 # nothing done yet: returns at once
    assert out == []
    gate.set()
    q.drain(block=True)
    assert out == [1, 2, 3, 4, 5] and len(q) == 0
    q.append((None, lambda: 1 / 0))
    time.sleep(0.05)
    with pytest.raises(ZeroDivisionError):
        q.drain(block=True)
    q.close()
    inline = _HostQueue(threaded=False)
    inline.append((None, lambda: out.append(6)))
    assert out[-1] == 5
    inline.drain()
    assert out[-1] == 6
