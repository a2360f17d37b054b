#!/bin/bash
# GPU-box routine: tests -> bench -> rocprofv3 kernel stats.  Every GPU step has
# its own time limit; a crash / timeout / abort ends the script (no retries).
# Test failures (exit 1) do not stop the bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; }
echo "== build" ; python -m stsphere.ops.build > $OUT/build.log 2>&1 || { echo build failed; cat $OUT/build.log; exit 2; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log
  if fatal $rc; then echo "pytest fatal rc=$rc"; exit $rc; fi
fi
echo "== bench"
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; tail -3 $OUT/bench.log
if [ $rc -ne 0 ]; then echo "bench rc=$rc"; exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 60 --warmup 6 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; tail -3 $OUT/prof.log
  if [ $rc -ne 0 ]; then echo "rocprof rc=$rc"; exit $rc; fi
fi
echo "== done"
