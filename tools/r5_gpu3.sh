#!/bin/bash
# round-5 GPU check 3: shared-GPU bench rows (ROWS="ranks:args;..."), then
# optionally the per-rank share proxies (SHARE="N:t:B ...").  A row that fails
# cleanly (exit 1) does not stop the script; a time limit or a crash does.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r5_c}
mkdir -p $OUT
cd $ROOT
i=0
IFS=';' read -ra ROWS_ <<< "${ROWS:-2:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5;6:--N 96 --tiles-per-edge 1 --steps 20 --warmup 5}"
for row in "${ROWS_[@]}"; do
  i=$((i + 1))
  n=${row%%:*}; args=${row#*:}
  STSP_SHARE_GPU=1 timeout -k 10 240 python -u bench.py --gpus $n $args --timeout 240 > $OUT/row$i.log 2>&1
  rc=$?
  echo "row $i ($n ranks, $args) rc=$rc"
  grep -E "^\[bench\]|^\{" $OUT/row$i.log | cut -c1-600 | tail -8
  [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
done
[ -n "$SHARE" ] && { TAG=${TAG:-r5_c} CONFIGS="$SHARE" bash tools/fused_share.sh || exit $?; }
echo "== all done"
