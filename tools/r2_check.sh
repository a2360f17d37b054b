#!/bin/bash
# Round-2 GPU check: GPU tests, driver-style bench runs, kernel stats.
# Every GPU step has its own limit; chained with && so a failure ends the call.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r2}
mkdir -p $OUT
cd $ROOT
run_tests() {
  [ "${SKIP_TESTS:-0}" = "1" ] && return 0
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  local rc=$?; tail -3 $OUT/pytest_gpu.log; return $rc
}
benches() {
  for i in 1 2; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench_20_5_$i.log 2>&1 || return $?
    tail -1 $OUT/bench_20_5_$i.log
  done
  timeout -k 10 200 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench_default.log 2>&1 || return $?
  tail -1 $OUT/bench_default.log
}
prof() {
  [ "${PROFILE:-1}" = "1" ] || return 0
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- \
    python3 $ROOT/bench.py --steps 60 --warmup 6 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  local rc=$?; cd $ROOT; return $rc
}
run_tests && benches && prof && echo "== done"
