#!/bin/bash
# round-5 GPU check: fused + solver GPU tests, fused probe + bench, shared-GPU
# rehearsals of BASELINE config 3 (C96, one panel per rank: 6 ranks; 3 ranks)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
TAG=r5_a TESTS="tests/test_fused.py tests/test_solver_gpu.py tests/test_native_runtime.py" ARMS="new:" REPS=3 bash tools/env_ab.sh || exit $?
mkdir -p gpurun_out/r5_a && timeout -k 10 180 python -u tools/ramp_probe.py > gpurun_out/r5_a/ramp.json 2> gpurun_out/r5_a/ramp.err || exit $?
cat gpurun_out/r5_a/ramp.json
TAG=r5_a ROWS="6:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5;3:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5" bash tools/rehearse.sh || exit $?
TAG=r5_a CONFIGS="90:1:18 48:2:8" bash tools/fused_share.sh || exit $?
echo "== all done"
