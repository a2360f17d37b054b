#!/bin/bash
# Last check of the round's tree: GPU suite, smoke, the driver-style bench.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_last}
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 3; }
grep smoke $OUT/smoke.log
for r in 1 2; do
  timeout -k 10 120 python -u bench.py > $OUT/bench_default_$r.log 2>&1 || exit $?
  tail -n 1 $OUT/bench_default_$r.log | cut -c1-230; echo
done
