#!/bin/bash
# round-5 GPU check 3: why the 6-rank C96 t=1 shared-GPU rehearsal timed out.
# One process first (t=1 loopback: the panel-per-rank ring protocol without
# other processes), then shared-GPU rows of growing rank count, then the
# per-rank share proxies.  A row that fails cleanly (exit 1) does not stop the
# script; a time limit or a crash does.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r5_c
mkdir -p $OUT
cd $ROOT
timeout -k 10 150 python -u tools/fused_probe.py --N 96 --t 1 --loopback --reps 5 > $OUT/probe_t1_loopback.json 2> $OUT/probe_t1_loopback.err
rc=$?; echo "t1 loopback probe rc=$rc"; tail -c 600 $OUT/probe_t1_loopback.json; tail -3 $OUT/probe_t1_loopback.err
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
i=0
for row in "2:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5" "3:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5" \
           "6:--N 96 --tiles-per-edge 2 --steps 20 --warmup 5" "6:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5"; do
  i=$((i + 1))
  n=${row%%:*}; args=${row#*:}
  STSP_SHARE_GPU=1 timeout -k 10 240 python -u bench.py --gpus $n $args --timeout 240 > $OUT/row$i.log 2>&1
  rc=$?
  echo "row $i ($n ranks, $args) rc=$rc"
  grep -E "^\[bench\]|^\{" $OUT/row$i.log | cut -c1-600 | tail -8
  [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
done
TAG=r5_c CONFIGS="90:1:18 48:2:8" bash tools/fused_share.sh || exit $?
echo "== all done"
