#!/bin/bash
# One-GPU C96: one tile per panel (tiles_per_edge 1: only panel-edge blocks
# push ghost copies) against the 24-tile decomposition (2), same box, interleaved.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-tpe}
mkdir -p $OUT
cd $ROOT
: > $OUT/bench.jsonl
for r in 1 2; do
  for t in 1 2; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --tiles-per-edge $t > $OUT/b_${t}_$r.log 2>&1 || { tail -5 $OUT/b_${t}_$r.log; exit 1; }
    grep '^{' $OUT/b_${t}_$r.log >> $OUT/bench.jsonl
    echo "t=$t 20/5: $(grep '^{' $OUT/b_${t}_$r.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"]*1e3,2))') us/step"
  done
done
for t in 1 2; do
  timeout -k 10 200 python -u bench.py --tiles-per-edge $t > $OUT/b_${t}_long.log 2>&1 || { tail -5 $OUT/b_${t}_long.log; exit 1; }
  grep '^{' $OUT/b_${t}_long.log >> $OUT/bench.jsonl
  echo "t=$t 300/30: $(grep '^{' $OUT/b_${t}_long.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"]*1e3,2))') us/step"
  timeout -k 10 120 python -u tools/kprobe.py --N 96 --t $t --blocks 16x16,16x8 > $OUT/k_$t.json 2>>$OUT/k.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/k_$t.json')); print('t=$t stage', {k:round(v['us_per_launch'],3) for k,v in d.items() if isinstance(v,dict)})"
done
