#!/bin/bash
# Throughput across grid sizes / dtypes / block shapes on one GPU (native
# runtime, graph replay).  Each run has its own limit; stop at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-sweep}
mkdir -p $OUT
cd $ROOT
: > $OUT/size_sweep.log
i=0
for v in "--N 96" "--N 96 --dtype fp32" "--N 180" "--N 360 --steps 100 --warmup 10" \
         "--N 720 --steps 40 --warmup 5" "--N 720 --steps 40 --warmup 5 --block 16x16" \
         "--N 720 --steps 40 --warmup 5 --dtype fp32" "--N 720 --steps 40 --warmup 5 --dtype fp32 --block 16x16"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py $v > $OUT/sz_$i.log 2>&1 || { tail -5 $OUT/sz_$i.log; exit 1; }
  echo "$v :: $(grep '^{' $OUT/sz_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), "us/step", "%.3e cell-updates/s" % d["value"], "block", d["config"].get("block"))')" | tee -a $OUT/size_sweep.log
done
