"""bench.py's transport chain between GPUs (xgmi -> ipc -> rccl) on one GPU
shared by two rank processes: with the direct rings refused
(STSP_FAIL_XGMI=1) the run lands on the graph-captured IPC copy transport,
replays every timed step from the graph and stays bitwise equal to one GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_falls_back_to_ipc_when_the_rings_fail():
    env = dict(os.environ, STSP_SHARE_GPU="1", STSP_FAIL_XGMI="1", OMP_NUM_THREADS="1",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--N", "48",
                        "--tiles-per-edge", "2", "--steps", "4", "--warmup", "2", "--timeout", "150"],
                       capture_output=True, text=True, timeout=200, env=env, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(lines[-1])
    assert out["status"] == "ok"
    assert out["config"]["comm"] == "ipc", out
    assert out["config"]["graph_replayed_steps"] == 4 and out["config"]["eager_steps"] == 0, out["config"]
    assert out["max_abs_diff_vs_1gpu_warmup"] == 0.0 and out["max_abs_diff_vs_1gpu"] == 0.0
    assert "STSP_FAIL_XGMI" in out["comm_fallback_reason"]
