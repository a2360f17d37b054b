#!/bin/bash
# fp32 two-columns-per-lane march (packed fp32) vs the one-column kernel: tests, C720 / C360 rows.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_march2}
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_march.py -v --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -12
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
run() {
  timeout -k 10 240 python -u bench.py --runtime native "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 4; }
  echo "$* :: $(tail -n 1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us/step", "%.3e" % d["value"])')" | tee -a $OUT/sizes.log
}
for m2 in 1 0; do
  for b in 64x4 64x8 64x16; do
    STSP_MARCH2=$m2 run --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype fp32 --block $b
  done
done
STSP_MARCH2=1 run --N 360 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype fp32 --block 64x4
STSP_MARCH2=1 run --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype fp64
STSP_MARCH2=1 run --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype fp32
echo "== done"
