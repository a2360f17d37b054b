#!/bin/bash
# Streaming-stage A/B at C720 on one GPU: the march GPU tests on the production
# build, then bench.py rows (fp64, fp32) per library variant, interleaved.
#   TAG=r5_march VARIANTS="prod <variant>" bash tools/march_ab.sh   (prod: the default library)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-march_ab}
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_march.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_march.log 2>&1
rc=$?; tail -2 $OUT/pytest_march.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for v in ${VARIANTS:-prod}; do
    sv=$v; [ "$v" = prod ] && sv=""
    for dt in fp64 fp32; do
      lab=${v}_${dt}_$rep
      STSP_VARIANT=$sv timeout -k 10 300 python -u bench.py --N 720 --tiles-per-edge 1 --dtype $dt --steps 10 --warmup 3 \
        > $OUT/bench_$lab.log 2> $OUT/bench_$lab.err || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,1), '%.3e' % d['value'], d['config'].get('runtime'), d['config'].get('block'))" $OUT/bench_$lab.log $lab
    done
  done
done
echo "== done"
