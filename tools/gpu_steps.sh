#!/bin/bash
# One GPU call as a list of named steps (replaces the per-round r5_*.sh
# scripts).  STEPS is "name=command;name=command;..." (commands run from the
# repo root); every step runs under its own `timeout -k 10 ${LIMIT:-300}` with
# its output in gpurun_out/$TAG/<name>.log.  A step that times out, aborts or
# crashes (rc 124/134/137/139 or > 128) ends the call; other failures are
# reported and the next step runs (no retries).  Example:
#   TAG=r6_x STEPS="tests=python -m pytest tests/test_march3.py -m gpu -q;bench=python bench.py --N 720 --tiles-per-edge 1 --steps 20 --warmup 5" bash tools/gpu_steps.sh
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-steps}
mkdir -p $OUT
cd $ROOT
IFS=';' read -ra steps <<< "${STEPS:?set STEPS=name=command;...}"
for s in "${steps[@]}"; do
  name=${s%%=*}; cmd=${s#*=}
  echo "== $name: $cmd"
  timeout -k 10 ${LIMIT:-300} bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  tail -${TAIL:-4} $OUT/$name.log
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "== $name: fatal rc=$rc, stopping"; exit $rc
  fi
  [ $rc -ne 0 ] && echo "== $name: rc=$rc"
done
echo "== all done"
