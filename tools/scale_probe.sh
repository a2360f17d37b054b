#!/bin/bash
# Larger grids on one GPU (bandwidth-bound regime), fp64 and fp32.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
python -m stsphere.ops.build --all > $OUT/build.log 2>&1 || exit 2
: > $OUT/bench_sizes.log
for v in "--N 180 --steps 200 --warmup 20" "--N 360 --steps 100 --warmup 10" "--N 720 --steps 40 --warmup 5" "--N 720 --steps 40 --warmup 5 --dtype fp32"; do
  timeout -k 10 400 python bench.py $v > $OUT/bench_tmp.log 2>&1 || { echo "bench failed: $v"; tail -5 $OUT/bench_tmp.log; exit 3; }
  echo "$v :: $(tail -1 $OUT/bench_tmp.log)" >> $OUT/bench_sizes.log
done
python3 -c "
import json
for l in open('$OUT/bench_sizes.log'):
    k, j = l.split(' :: ', 1); d = json.loads(j)
    print(f'{k:45s} {d[\"value\"]:.3e} cups  {d[\"ms_per_step\"]:.3f} ms/step finite={d[\"finite\"]}')
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/pmc_c720 -o k --output-format csv -- python3 $ROOT/bench.py --N 720 --steps 6 --warmup 2 > $OUT/pmc_c720.log 2>&1 || { echo "pmc failed"; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c720 -o k --output-format csv -- python3 $ROOT/bench.py --N 720 --steps 20 --warmup 2 > $OUT/prof_c720.log 2>&1 || { echo "prof failed"; exit 5; }
echo done
