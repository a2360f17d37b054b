#!/bin/bash
# HIP runtime knobs against the driver-style C96 bench (20 timed steps, one
# graph replay): graph packet capture, device kernargs, host wait mode.
# Unknown variables are ignored by the runtime; each run has its own limit.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-envab}
mkdir -p $OUT
cd $ROOT
: > $OUT/summary.txt
i=0
for r in 1 2; do
for v in "NONE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0" \
         "HIP_FORCE_DEV_KERNARG=1" "ROC_ACTIVE_WAIT_TIMEOUT=1000" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"; do
  i=$((i+1))
  env $v timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/b_$i.log 2>&1 || { tail -5 $OUT/b_$i.log; exit 1; }
  echo "$v :: $(grep '^{' $OUT/b_$i.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"]*1e3,2))') us/step" | tee -a $OUT/summary.txt
done
done
