#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r3_c180
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for v in "--N 180 --tiles-per-edge 3 --runtime fused" "--N 180 --tiles-per-edge 2 --runtime fused" "--N 180 --tiles-per-edge 3 --runtime native"; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 $v > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 4; }
  echo "$v :: $(tail -n 1 $OUT/b.log | cut -c1-330)" | tee -a $OUT/c180.log
done
timeout -k 10 200 python -u tools/launch_probe.py --N 96 --t 2 --steps 20 --reps 30 > $OUT/launch_probe.json 2> $OUT/launch_probe.err || { tail -5 $OUT/launch_probe.err; exit 5; }
cat $OUT/launch_probe.json
