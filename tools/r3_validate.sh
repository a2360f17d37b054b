#!/bin/bash
# Round-3 validation on one GPU: the whole GPU test suite, smoke, the
# driver-style bench (20/5, twice) and a 300/30 run, rocprofv3 kernel stats of
# the 20/5 bench, the C180 and C720 rows.  Every GPU step has its own limit;
# the script stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_val}
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log | grep smoke
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_20_5_$r.log 2>&1 || exit $?
  tail -n 1 $OUT/bench_20_5_$r.log | cut -c1-300; echo
done
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > $OUT/bench_300_30.log 2>&1 || exit $?
tail -n 1 $OUT/bench_300_30.log | cut -c1-300; echo
for v in "--N 180 --steps 20 --warmup 5 --runtime fused" "--N 180 --steps 20 --warmup 5 --runtime native" \
         "--N 720 --steps 10 --warmup 2 --runtime fused" "--N 720 --steps 10 --warmup 2 --runtime native" \
         "--N 720 --steps 10 --warmup 2 --dtype fp32 --runtime native"; do
  timeout -k 10 240 python -u bench.py $v > $OUT/sz.log 2>&1 || { tail -5 $OUT/sz.log; exit 4; }
  echo "$v :: $(tail -n 1 $OUT/sz.log | cut -c1-400)" >> $OUT/sizes.log
done
cat $OUT/sizes.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- \
  python3 $ROOT/bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
echo "== done"
