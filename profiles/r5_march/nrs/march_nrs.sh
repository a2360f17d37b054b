#!/bin/bash
# Streaming-stage job count at C720 on one GPU: the march GPU tests, then
# bench.py rows with STSP_MARCH_NRS (row segments per strip; 0 = ceil(n / 4)),
# interleaved.   NRS="0 170 ..." DTYPES="fp64 fp32" bash tools/march_nrs.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-march_nrs}
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_march.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_march.log 2>&1
rc=$?; tail -2 $OUT/pytest_march.log; [ $rc = 0 ] || exit $rc
for rep in ${REPS:-1 2}; do
  for dt in ${DTYPES:-fp64 fp32}; do
    for nrs in ${NRS:-0 170}; do
      lab=${dt}_nrs${nrs}_$rep
      STSP_MARCH_NRS=$nrs timeout -k 10 300 python -u bench.py --N ${N:-720} --tiles-per-edge 1 --dtype $dt --steps 10 --warmup 3 \
        > $OUT/bench_$lab.log 2> $OUT/bench_$lab.err || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,1), '%.3e' % d['value'], d['config'].get('runtime'), d['config'].get('block'), d.get('finite'))" $OUT/bench_$lab.log $lab
    done
  done
done
echo "== done"
