#!/bin/bash
# Streaming stage: own-row operands one row ahead (PF) vs not.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_pf}
mkdir -p $OUT
cd $ROOT
STSP_MARCH_PF=1 timeout -k 10 400 python -u -m pytest tests/test_march.py -v --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; grep -E "^E +assert|FAILED|passed|failed" $OUT/pytest.log | tail -8
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
for cg in 1 0; do
  for dt in fp64 fp32; do
    for b in 64x4 64x8; do
      STSP_MARCH_PF=$cg timeout -k 10 200 python -u bench.py --runtime native --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype $dt --block $b > $OUT/b.log 2>&1 || { tail -3 $OUT/b.log; exit 4; }
      echo "pf=$cg $dt $b :: $(tail -n 1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us/step", "%.3e" % d["value"])')" | tee -a $OUT/sizes.log
    done
  done
done
