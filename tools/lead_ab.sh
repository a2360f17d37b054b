#!/bin/bash
# Short first graph (--lead-steps L) against one graph for the 20 timed steps,
# with kernel arguments in device memory (default) or host memory.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-lead}
mkdir -p $OUT
cd $ROOT
: > $OUT/summary.txt
i=0
for r in 1 2; do
for ka in dflt 0; do
for L in 0 1 2 3 4; do
  i=$((i+1))
  envv="NONE=1"; [ $ka = 0 ] && envv="HIP_FORCE_DEV_KERNARG=0"
  env $envv timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --lead-steps $L > $OUT/b_$i.log 2>&1 || { tail -5 $OUT/b_$i.log; exit 1; }
  echo "kernarg=$ka lead=$L :: $(grep '^{' $OUT/b_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), d["config"]["graph_replayed_steps"], d["max_abs_diff_vs_1gpu"])') us/step" | tee -a $OUT/summary.txt
done
done
done
