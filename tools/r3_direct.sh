#!/bin/bash
# Headline bench with direct fused launches (default) vs graph replay, and the TT kernel tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_direct}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_tt_kernels.py -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_tt.log 2>&1; rc=$?; grep -E "FAILED|passed|failed" $OUT/pytest_tt.log | tail -5; [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
for r in 1 2 3; do
  for l in direct graph; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --launch $l > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 4; }
    echo "$l $r :: $(tail -n 1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["ms_per_step"]*1e3,2), "us/step", "%.3e" % d["value"], c["direct_launch_steps"], c["kernel_launches"], c["graph_replayed_steps"])')" | tee -a $OUT/bench.log
  done
done
cp $OUT/b.log $OUT/bench_last.json
echo "== done"
