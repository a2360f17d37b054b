#!/bin/bash
# round-5 GPU check 2: persistent TT step (tests + probe), the host cost of a
# timed region, and last the standalone uncached-memory reproducer
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r5_b
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_tt_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k persistent > $OUT/pytest_tt.log 2>&1; rc=$?; tail -3 $OUT/pytest_tt.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u tools/tt_persist_probe.py > $OUT/tt_persist.json 2> $OUT/tt_persist.err || exit $?
cat $OUT/tt_persist.json
timeout -k 10 120 python -u tools/launch_overhead.py > $OUT/launch_overhead.json 2> $OUT/launch_overhead.err || exit $?
cat $OUT/launch_overhead.json
# C720 on one GPU: the fused step, one launch per step (not resident), against the streaming stage
for cfg in fp64:20 fp64:16 fp32:20; do
  dt=${cfg%%:*}; B=${cfg##*:}
  timeout -k 10 420 python -u bench.py --N 720 --tiles-per-edge 1 --runtime fused --block $B --dtype $dt --steps 10 --warmup 3 > $OUT/c720_fused_${dt}_B$B.json 2> $OUT/c720_fused_${dt}_B$B.err || exit $?
  cat $OUT/c720_fused_${dt}_B$B.json
done
timeout -k 10 120 ./tools/ring_repro 60 4 > $OUT/ring_repro.json 2> $OUT/ring_repro.err; echo "ring_repro rc=$?"; cat $OUT/ring_repro.json
echo "== all done"
