#!/bin/bash
# In-launch hand-off A/B of the one-rank multi-step fused launch
# (STSP_FUSED_HANDOFF=epoch: write-through state, drained per-block step
# counter, producer poll; =tag: tagged granules, the data is the flag):
# fused GPU tests under the candidate, then interleaved in-kernel probes and
# driver-style benches.
#   TAG=r6_handoff bash tools/handoff_ab.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r6_handoff}
mkdir -p $OUT
cd $ROOT
STSP_FUSED_HANDOFF=tag timeout -k 10 400 python -u -m pytest tests/test_fused.py tests/test_long_run.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $OUT/pytest_tag.log 2>&1 || { tail -30 $OUT/pytest_tag.log; exit 1; }
tail -2 $OUT/pytest_tag.log
for rep in 1 2 3; do
  for m in epoch tag; do
    STSP_FUSED_HANDOFF=$m timeout -k 10 120 python -u tools/fused_probe.py --N 96 --t 2 > $OUT/probe_C96_${m}_$rep.json 2> $OUT/probe_C96_${m}_$rep.err || exit $?
    STSP_FUSED_HANDOFF=$m timeout -k 10 120 python -u tools/fused_probe.py --N 36 --t 1 --B 6 > $OUT/probe_C36B6_${m}_$rep.json 2> $OUT/probe_C36B6_${m}_$rep.err || exit $?
    STSP_FUSED_HANDOFF=$m timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_${m}_$rep.json 2> $OUT/bench_${m}_$rep.err || exit $?
    python - $OUT $m $rep <<'PY'
import json, sys
out, m, rep = sys.argv[1:]
last = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
a = last(f"{out}/probe_C96_{m}_{rep}.json"); b = last(f"{out}/probe_C36B6_{m}_{rep}.json"); c = last(f"{out}/bench_{m}_{rep}.json")
print(m, rep, "C96 multi20/100 %.2f/%.2f" % (a["multi20_us_per_step"], a["multi100_us_per_step"]),
      "| C36B6 multi100 %.2f" % b["multi100_us_per_step"], "| bench 20/5 %.2f us" % (c["ms_per_step"] * 1e3))
PY
  done
done
echo "== handoff_ab done"
