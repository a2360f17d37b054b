#!/bin/bash
# GPU box: full GPU tests, the TT benchmark, its kernel stats and the MFMA counters.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tt_bench.py --json $OUT/tt_bench.json > $OUT/tt_bench.log 2>&1 || { tail $OUT/tt_bench.log; exit 3; }
cat $OUT/tt_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ttprof -o tt --output-format csv -- python3 $ROOT/tools/tt_bench.py --sizes 4096,16384 --steps 10 > $OUT/ttprof.log 2>&1 || { tail $OUT/ttprof.log; exit 4; }
echo "== stats"; find $OUT/ttprof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-6 | head -14
