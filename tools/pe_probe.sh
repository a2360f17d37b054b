#!/bin/bash
# Panel-edge phase cost at C96 (and C720): graph-timed stage launches with and
# without the panel-edge bits, then the driver-style bench.  Each GPU step has
# its own limit; the chain stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-pe}
mkdir -p $OUT
cd $ROOT
timeout -k 10 200 python -u tools/kprobe.py --blocks ${BLOCKS:-16x16} > $OUT/kprobe.json 2> $OUT/kprobe.err &&
timeout -k 10 200 python -u tools/kprobe.py --blocks ${BLOCKS:-16x16} --no-pedge > $OUT/kprobe_nope.json 2>> $OUT/kprobe.err &&
python -c "
import json
a=json.load(open('$OUT/kprobe.json')); b=json.load(open('$OUT/kprobe_nope.json'))
for k,v in a.items():
    if isinstance(v,dict): print(k,'pedge',round(v['us_per_launch'],3),'no-pedge',round(b[k]['us_per_launch'],3))
print('tiny',round(a['tiny_kernel_us_per_launch'],3))
" &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.log 2>&1 && tail -1 $OUT/bench_20_5.log | cut -c1-200 &&
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > $OUT/bench_300.log 2>&1 && tail -1 $OUT/bench_300.log | cut -c1-200
