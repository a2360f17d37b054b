#!/bin/bash
# Environment A/B on one GPU box: optional GPU tests, then for every arm of
# ARMS (space-separated "label:VAR=value[,VAR=value]" or "label:" for the
# defaults) tools/fused_probe.py (launch rates, per-block phase stamps), then
# the driver-style bench interleaved over the arms (REPS rounds), so box drift
# hits every arm alike.  Every GPU step has its own time limit; the first
# failure ends the script.
#   TAG=r5_sched ARMS="new: legacy:STSP_FUSED_SCHED=legacy" tools/env_ab.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-env_ab}
mkdir -p $OUT
cd $ROOT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -4 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
fi
arm_env() {   # "label:A=1,B=2" -> "A=1 B=2"
  local spec=${1#*:}
  echo ${spec//,/ }
}
for arm in ${ARMS:-base:}; do
  lab=${arm%%:*}
  if [ "${PROBE:-1}" = "1" ]; then
    env $(arm_env $arm) timeout -k 10 240 python -u tools/fused_probe.py --N ${N:-96} --t ${T:-2} ${PROBE_ARGS:---stamps} \
      > $OUT/probe_$lab.json 2> $OUT/probe_$lab.err || exit $?
    python - "$OUT/probe_$lab.json" "$lab" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["graph_us_per_step", "multi20_us_per_step", "multi100_us_per_step", "host_timed_20_us_per_step"]
print(sys.argv[2], {k: d.get(k) for k in keys})
m = d.get("multi_last_step_cycles")
if m:
    print("   last step:", {k: (v["int"], v["edge"], v["corner"]) for k, v in m.items()})
EOF
  fi
done
for i in $(seq 1 ${REPS:-2}); do
  for arm in ${ARMS:-base:}; do
    lab=${arm%%:*}
    env $(arm_env $arm) timeout -k 10 120 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS:-} \
      > $OUT/bench_${lab}_$i.log 2>&1 || exit $?
    tail -n 1 $OUT/bench_${lab}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lab', {k: d.get(k) for k in ('value','ms_per_step')})"
  done
done
echo "== done"
