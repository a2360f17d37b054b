#!/bin/bash
# The streaming SWE stage (march_kernel.hip): GPU tests, then C720 / C360 / C180
# bench rows, block stage kernel vs march row counts, fp64 and fp32.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_march}
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_march.py -v --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -12
# test failures (rc 1) still let the timing rows run; a crash, abort or time limit ends the script
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
run() {
  timeout -k 10 240 python -u bench.py --runtime native "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 4; }
  echo "$* :: $(tail -n 1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us/step", "%.3e" % d["value"])')" | tee -a $OUT/sizes.log
}
for dt in fp64 fp32; do
  for b in 64x4 64x8 64x16 ""; do
    run --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype $dt ${b:+--block $b}
  done
done
for b in 64x4 64x8 ""; do run --N 360 --tiles-per-edge 1 --steps 10 --warmup 2 ${b:+--block $b}; done
for b in 64x4 64x8 ""; do run --N 180 --tiles-per-edge 1 --steps 20 --warmup 5 ${b:+--block $b}; done
echo "== done"
