#!/bin/bash
# Persistent step kernel: GPU tests, then A/B against graph replay at C96.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-persist}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_native_runtime.py -x -v --timeout 120 --timeout-method thread \
  -k "persistent" > $OUT/pytest_persist.log 2>&1
rc=$?; tail -15 $OUT/pytest_persist.log; [ $rc -eq 0 ] || exit $rc
for args in "--runtime native" "--runtime persistent --block 16x16" "--runtime persistent --block 16x16 --tiles-per-edge 1" ; do
  for st in "--steps 20 --warmup 5" "--steps 300 --warmup 30"; do
    timeout -k 10 120 python -u bench.py $args $st > $OUT/b.log 2>&1 || { cat $OUT/b.log; exit 1; }
    echo "$args $st :: $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/b.log') if l.startswith('{')][0]); print(round(d['ms_per_step']*1e3,2), 'us/step', '%.3e'%d['value'])")"
  done
done
