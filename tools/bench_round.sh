#!/bin/bash
# 1-GPU bench variants + rocprofv3 kernel stats of the default bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
python -m stsphere.ops.build --all > $OUT/build.log 2>&1 || exit 2
for v in "--runtime persistent" "--runtime native" "--runtime persistent --dtype fp32" "--runtime persistent --tiles-per-edge 1" "--runtime native --N 720 --steps 40 --warmup 4"; do
  timeout -k 10 240 python bench.py --steps 600 --warmup 60 $v > $OUT/bench_tmp.log 2>&1 || { echo "bench failed: $v"; tail -5 $OUT/bench_tmp.log; exit 3; }
  echo "$v :: $(tail -1 $OUT/bench_tmp.log)" >> $OUT/bench_variants.log
done
cat $OUT/bench_variants.log | python3 -c "
import sys, json
for l in sys.stdin:
    k, j = l.split(' :: ', 1)
    d = json.loads(j)
    print(f'{k:45s} {d[\"value\"]:.3e} cups  {1e3*d[\"ms_per_step\"]:.2f} us/step  sdpd={d[\"simulated_days_per_day\"]:.3e} finite={d[\"finite\"]}')
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 200 --warmup 20 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 4; }
echo done
