#!/bin/bash
# Fused kernel iteration: GPU tests of the fused step, then the timing / stamp probe.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_fq}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_fused.log 2>&1; rc=$?; tail -3 $OUT/pytest_fused.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u tools/fused_probe.py --N ${N:-96} --t ${T:-2} --stamps --stage ${PROBE_ARGS:-} \
  > $OUT/probe.json 2> $OUT/probe.err || { tail -5 $OUT/probe.err; exit 3; }
cat $OUT/probe.json
