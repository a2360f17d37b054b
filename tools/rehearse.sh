#!/bin/bash
# Shared-GPU rehearsals of the multi-rank bench paths on a one-GPU box
# (STSP_SHARE_GPU=1: every rank on cuda:0, gloo between processes, the
# direct xGMI rings through same-GPU IPC).  Each row: ranks and bench
# arguments; the JSON line of rank 0 goes to $OUT/<tag>.json.
#   TAG=r4_rehearse ROWS="8:--N 720 --tiles-per-edge 2 --dtype fp32 --block 64x4" tools/rehearse.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-rehearse}
mkdir -p $OUT
cd $ROOT
IFS=';' read -ra rows <<< "${ROWS:-8:--N 720 --tiles-per-edge 2 --dtype fp32 --block 64x4 --steps 4 --warmup 2}"
i=0
for row in "${rows[@]}"; do
  n=${row%%:*}
  args=${row#*:}
  i=$((i + 1))
  STSP_SHARE_GPU=1 timeout -k 10 ${ROW_TIMEOUT:-300} python -u bench.py --gpus $n $args --timeout ${ROW_TIMEOUT:-300} \
    > $OUT/row$i.log 2>&1 || { echo "row $i failed: $row"; tail -5 $OUT/row$i.log; exit 1; }
  tail -n 1 $OUT/row$i.log > $OUT/row$i.json
  echo "row $i ($n ranks, $args):"; cut -c1-400 $OUT/row$i.json; echo
done
echo "== done"
