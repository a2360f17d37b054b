#!/bin/bash
# Epoch hand-off of the one-rank multi-step fused launch: wave 0 polls every
# producer of the block before a barrier (STSP_FUSED_POLL=block) or each ring
# thread polls its own cell's producer and loads at once (cell).  Fused GPU
# tests under the candidate, then interleaved in-kernel probes and
# driver-style benches.   TAG=r6_poll bash tools/poll_ab.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r6_poll}
mkdir -p $OUT
cd $ROOT
STSP_FUSED_POLL=cell timeout -k 10 400 python -u -m pytest tests/test_fused.py tests/test_long_run.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $OUT/pytest_cell.log 2>&1 || { tail -30 $OUT/pytest_cell.log; exit 1; }
tail -2 $OUT/pytest_cell.log
for rep in 1 2 3; do
  for m in block cell; do
    STSP_FUSED_POLL=$m timeout -k 10 120 python -u tools/fused_probe.py --N 96 --t 2 > $OUT/probe_C96_${m}_$rep.json 2> $OUT/probe_C96_${m}_$rep.err || exit $?
    STSP_FUSED_POLL=$m timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_${m}_$rep.json 2> $OUT/bench_${m}_$rep.err || exit $?
    python - $OUT $m $rep <<'PY'
import json, sys
out, m, rep = sys.argv[1:]
last = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
a = last(f"{out}/probe_C96_{m}_{rep}.json"); c = last(f"{out}/bench_{m}_{rep}.json")
print(m, rep, "C96 multi20/100 %.2f/%.2f" % (a["multi20_us_per_step"], a["multi100_us_per_step"]),
      "| bench 20/5 %.2f us" % (c["ms_per_step"] * 1e3))
PY
  done
done
echo "== poll_ab done"
