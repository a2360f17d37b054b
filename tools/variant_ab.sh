#!/bin/bash
# Fused-step A/B of library variants on one box, interleaved: the fused GPU
# tests on the candidate, then per rep and variant the in-kernel probe
# (no stamps) and the driver-style bench.
#   TAG=r5_prio VARIANTS="prod prio" REPS="1 2 3" bash tools/variant_ab.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-variant_ab}
mkdir -p $OUT
cd $ROOT
CAND=${CAND:-${VARIANTS##* }}
STSP_VARIANT=$CAND timeout -k 10 400 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/pytest_$CAND.log 2>&1; rc=$?; tail -2 $OUT/pytest_$CAND.log; [ $rc = 0 ] || exit $rc
for rep in ${REPS:-1 2 3}; do
  for v in ${VARIANTS:-prod}; do
    [ "$v" = prod ] && vv="" || vv=$v
    STSP_VARIANT=$vv timeout -k 10 180 python -u tools/fused_probe.py --N 96 --t 2 > $OUT/probe_${v}_$rep.json 2> $OUT/probe_${v}_$rep.err || exit $?
    STSP_VARIANT=$vv timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_${v}_$rep.log 2> $OUT/bench_${v}_$rep.err || exit $?
    python3 - $OUT/probe_${v}_$rep.json $OUT/bench_${v}_$rep.log ${v}_$rep <<'PY'
import json, sys
p = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "multi100", p.get("multi100_us_per_step"), "multi20", p.get("multi20_us_per_step"),
      "bench", round(b["ms_per_step"] * 1e3, 2), "%.3e" % b["value"])
PY
  done
done
echo "== done"
