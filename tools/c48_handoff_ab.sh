#!/bin/bash
# C48 on one GPU (BASELINE config 2; fused B = 8 blocks): epoch vs tagged
# in-launch hand-off, three interleaved reps of the in-kernel probe and the
# driver-style bench.   TAG=r6_c48 bash tools/c48_handoff_ab.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r6_c48}
mkdir -p $OUT
cd $ROOT
for rep in 1 2 3; do
  for m in epoch tag; do
    STSP_FUSED_HANDOFF=$m timeout -k 10 120 python -u tools/fused_probe.py --N 48 --t 1 > $OUT/probe_${m}_$rep.json 2> $OUT/probe_${m}_$rep.err || exit $?
    STSP_FUSED_HANDOFF=$m timeout -k 10 180 python -u bench.py --gpus 1 --N 48 --tiles-per-edge 1 --steps 20 --warmup 5 > $OUT/bench_${m}_$rep.json 2> $OUT/bench_${m}_$rep.err || exit $?
    python - $OUT $m $rep <<'PY'
import json, sys
out, m, rep = sys.argv[1:]
last = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
a = last(f"{out}/probe_{m}_{rep}.json"); c = last(f"{out}/bench_{m}_{rep}.json")
print(m, rep, "B", a["B"], "C48 multi20/100 %.2f/%.2f" % (a["multi20_us_per_step"], a["multi100_us_per_step"]),
      "| bench 20/5 %.2f us" % (c["ms_per_step"] * 1e3), c["config"].get("fused_block"))
PY
  done
done
echo "== c48 done"
