#!/bin/bash
# Kernel A/B on the GPU box: HIP numerics tests of the production build, then
# per library variant (VARIANTS; "prod" = production) the graph-timed stage
# launch (kprobe) and the 1-GPU bench; stamp builds (STAMPS) give phase timelines.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_native_runtime.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread > $OUT/ab_pytest.log 2>&1
rc=$?; tail -3 $OUT/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-prod}; do
  [ "$v" = prod ] && export STSP_VARIANT= || export STSP_VARIANT=$v
  timeout -k 10 200 python tools/kprobe.py --blocks ${BLOCKS:-16x16} ${KPROBE_ARGS:-} > $OUT/ab_kprobe_$v.json 2>$OUT/ab_kprobe_$v.err || exit $?
  timeout -k 10 200 python bench.py --steps 600 --warmup 60 ${BENCH_ARGS:-} > $OUT/ab_bench_$v.log 2>&1 || exit $?
  echo "$v kprobe: $(python3 -c "import json; a=json.load(open('$OUT/ab_kprobe_$v.json')); print({k: round(v['us_per_launch'],3) for k,v in a.items() if isinstance(v,dict)})") bench: $(grep -h '^{' $OUT/ab_bench_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(1e3*d['ms_per_step'],2), 'us/step', '%.3e' % d['value'])")"
done
for v in ${STAMPS:-}; do
  STSP_VARIANT=$v timeout -k 10 200 python tools/kprobe.py --stamps --blocks 16x16 ${KPROBE_ARGS:-} > $OUT/ab_stamps_$v.json 2>$OUT/ab_stamps_$v.err || exit $?
  python3 -c "import json; b=json.load(open('$OUT/ab_stamps_$v.json')); print('$v', json.dumps(b['16x16'].get('wave_stamp_cycles_median')))"
done
echo "== done"
