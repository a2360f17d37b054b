#!/bin/bash
# round-5 final-tree check, part 1: the whole GPU suite
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r5_final}
mkdir -p $OUT
cd $ROOT
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; exit $rc
