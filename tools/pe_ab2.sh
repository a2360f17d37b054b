#!/bin/bash
# Same-box A/B at C96 16x16: production vs the pre-panel-edge library
# (libstsp_prepe.so, commit d318046: index-space ghosts, no interpolation;
# timing only) vs production with the panel-edge bits cleared; then tests and
# the driver-style bench.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-peab}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_native_runtime.py -x -q --timeout 120 \
   --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in prod prepe nope prod2 prepe2; do
  case $v in
    prod|prod2) timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 > $OUT/k_$v.json 2>> $OUT/k.err || exit $? ;;
    prepe|prepe2) STSP_VARIANT=prepe timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 > $OUT/k_$v.json 2>> $OUT/k.err || exit $? ;;
    nope) timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 --no-pedge > $OUT/k_$v.json 2>> $OUT/k.err || exit $? ;;
  esac
done
python -c "
import json
for v in ['prod','prepe','nope','prod2','prepe2']:
    a=json.load(open('$OUT/k_'+v+'.json'))
    print(v, round(a['16x16']['us_per_launch'],3), 'tiny', round(a['tiny_kernel_us_per_launch'],3))
" &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.log 2>&1 && tail -1 $OUT/bench_20_5.log | cut -c1-230 &&
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > $OUT/bench_300.log 2>&1 && tail -1 $OUT/bench_300.log | cut -c1-230
