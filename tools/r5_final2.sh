#!/bin/bash
# round-5 final-tree check, part 2: smoke, the driver-style bench, and a
# rocprofv3 kernel-trace summary of the same bench
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r5_final}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_$i.log 2> $OUT/bench_$i.err || exit $?
  tail -1 $OUT/bench_$i.log | cut -c1-200
done
timeout -k 10 180 python -u bench.py > $OUT/bench_default.log 2> $OUT/bench_default.err || exit $?
tail -1 $OUT/bench_default.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name "*kernel_stats*" | head -3
echo "== done"
