"""bench.py contract on the CPU (torch backend, gloo): the self-launching
multi-rank entry point and the one-rank JSON line."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_one_rank_cpu():
    out = _run(["--backend", "torch", "--N", "12", "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert out["metric"] == "cell-updates/sec (whole node) at C12"
    assert out["value"] > 0 and out["finite"] and out["higher_is_better"] is True
    assert out["max_abs_diff_vs_1gpu"] is None


@pytest.mark.parametrize("gpus,t", [(2, 1), (3, 1)])
def test_bench_self_launches_ranks_cpu(gpus, t):
    """--gpus N without torchrun spawns N ranks; the warmup state and the final
    state must equal one rank's bit for bit."""
    out = _run(["--gpus", str(gpus), "--backend", "torch", "--N", "12", "--tiles-per-edge", str(t),
                "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == gpus
    assert out["max_abs_diff_vs_1gpu_warmup"] == 0.0 and out["max_abs_diff_vs_1gpu"] == 0.0
    assert out["config"]["comm"] == "torch.distributed"


def test_bench_deadline_kills_hung_rank_cpu():
    """A rank that never returns (test hook) is killed at --timeout: the parent
    prints one status=timeout JSON line naming each rank's last phase and exits
    non-zero, well inside the driver's own limit."""
    import time
    env = dict(os.environ, OMP_NUM_THREADS="1", STSP_BENCH_HANG_RANK="1")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "torch",
                        "--N", "12", "--steps", "2", "--warmup", "1", "--timeout", "25"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode != 0
    assert time.time() - t0 < 120
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr
    out = json.loads(lines[0])
    assert out["status"] == "timeout" and out["value"] is None
    # phases carry the transport being tried (warmup_<comm>, verify_<comm>)
    assert out["phases"]["1"]["phase"].startswith("warmup")
    assert out["phases"]["0"]["phase"].split("_")[0] in ("warmup", "verify")


def test_bench_preflight_refuses_missing_gpus():
    """--gpus N on the HIP backend with fewer visible GPUs: one status=error
    line, no ranks started (this container has no GPU at all)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs visible")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("STSP_SHARE_GPU", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["status"] == "error" and "GPU" in out["error"]
