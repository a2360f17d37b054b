#!/bin/bash
# Fused-step A/B on one GPU box: GPU tests of the fused kernel (production
# library), then tools/fused_probe.py (launch rates, per-block phase stamps)
# for every library variant named in VARIANTS ("" = production), then the
# driver-style bench.  Every GPU step has its own time limit; the first
# failure ends the script.
#   TAG=r4_ho VARIANTS="prod ho0 early0" tools/fused_ab.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-fused_ab}
mkdir -p $OUT
cd $ROOT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest ${TESTS:-tests/test_fused.py} -m gpu -x -v --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -4 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
fi
for v in ${VARIANTS:-prod}; do
  [ "$v" = prod ] && vv="" || vv=$v
  STSP_VARIANT=$vv timeout -k 10 180 python -u tools/fused_probe.py --N ${N:-96} --t ${T:-2} ${PROBE_ARGS:---stamps} \
    > $OUT/probe_$v.json 2> $OUT/probe_$v.err || exit $?
  python - "$OUT/probe_$v.json" "$v" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["graph_us_per_step", "multi20_us_per_step", "multi100_us_per_step", "host_timed_20_us_per_step"]
print(sys.argv[2], {k: d.get(k) for k in keys})
m = d.get("multi_last_step_cycles")
if m:
    print("   last step:", {k: (v["int"], v["edge"], v["corner"]) for k, v in m.items()})
EOF
done
if [ "${BENCH:-1}" = "1" ]; then
  for i in 1 2; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > $OUT/bench_20_5_$i.log 2>&1 || exit $?
    tail -n 1 $OUT/bench_20_5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','repeat_ms_per_step')}, d['config'].get('host_sync'))"
  done
fi
echo "== done"
