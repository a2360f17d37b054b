#!/bin/bash
# Round-3 fused-step check: GPU tests of the fused kernel, driver-style bench
# (fused vs launch-per-stage), multi-rank rehearsals sharing the GPU, kernel stats.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_fused}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_fused.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_fused.log 2>&1; rc=$?; tail -4 $OUT/pytest_fused.log; [ $rc = 0 ] || exit $rc
for rt in fused native fused; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --runtime $rt > $OUT/bench_20_5_$rt.log 2>&1 || exit $?
  tail -n 1 $OUT/bench_20_5_$rt.log | cut -c1-420
done
timeout -k 10 200 python -u bench.py --runtime fused > $OUT/bench_300_fused.log 2>&1 || exit $?
tail -n 1 $OUT/bench_300_fused.log | cut -c1-300
for g in 2 8; do
  STSP_SHARE_GPU=1 timeout -k 10 200 python -u bench.py --gpus $g --steps 20 --warmup 5 --timeout 150 \
    > $OUT/rehearsal_$g.log 2>&1 || exit $?
  tail -n 1 $OUT/rehearsal_$g.log | cut -c1-300; echo
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- \
  python3 $ROOT/bench.py --steps 60 --warmup 6 --runtime fused > $OUT/prof.log 2>&1 || exit $?
echo "== done"
