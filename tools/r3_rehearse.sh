#!/bin/bash
# Shared-GPU rehearsals through the bench entry point (ranks on one GPU, correctness only):
# the fused multi-step path with direct launches at 2 and 8 ranks (C96), and 8 ranks at C180.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_rehearse}
mkdir -p $OUT
cd $ROOT
for v in "--gpus 2" "--gpus 8" "--gpus 8 --N 180" "--gpus 2 --launch direct"; do
  tag=$(echo $v | tr -d ' -')
  STSP_SHARE_GPU=1 timeout -k 10 250 python -u bench.py $v --steps 20 --warmup 5 --timeout 200 > $OUT/rehearsal_$tag.log 2>&1 || { tail -5 $OUT/rehearsal_$tag.log; exit 4; }
  echo "$v :: $(tail -n 1 $OUT/rehearsal_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["status"], c["runtime"], c["comm"], "diff_warm", d["max_abs_diff_vs_1gpu_warmup"], "diff_final", d["max_abs_diff_vs_1gpu"], "launches", c.get("kernel_launches"), "direct", c.get("direct_launch_steps"))')" | tee -a $OUT/summary.log
done
