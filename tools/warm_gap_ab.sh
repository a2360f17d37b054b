#!/bin/bash
# Driver-style bench with and without the synchronize right after the warm-up
# (STSP_BENCH_WARM_SYNC=1: round 5's order, the GPU idles ~50 us before the
# timed launch), interleaved.   TAG=r6_warm bash tools/warm_gap_ab.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r6_warm}
mkdir -p $OUT
cd $ROOT
for rep in 1 2 3 4; do
  for m in 1 0; do
    STSP_BENCH_WARM_SYNC=$m timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_sync${m}_$rep.json 2> $OUT/bench_sync${m}_$rep.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('warm_sync=' + sys.argv[2], sys.argv[3], '%.2f us/step' % (d['ms_per_step'] * 1e3))" $OUT/bench_sync${m}_$rep.json $m $rep
  done
done
echo "== warm_gap_ab done"
