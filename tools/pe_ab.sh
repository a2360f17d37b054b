#!/bin/bash
# A/B of the panel-edge fix-up at C96 16x16: production (border-wave fix-up,
# STSP_PE_WAVE=1) vs the block-wide fix-up (variant pe0) vs no panel edges
# (timing only), then the HIP numerics tests on the production library and the
# driver-style bench.  Every GPU step has its own limit; the chain stops at the
# first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-peab}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_native_runtime.py -x -q --timeout 120 \
   --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 > $OUT/k_pew.json 2> $OUT/k.err &&
STSP_VARIANT=pe0 timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 > $OUT/k_pe0.json 2>> $OUT/k.err &&
timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 --no-pedge > $OUT/k_nope.json 2>> $OUT/k.err &&
timeout -k 10 200 python -u tools/kprobe.py --stamps --blocks 16x16 > $OUT/s_pew.json 2>> $OUT/k.err &&
python -c "
import json
for v in ['pew','pe0','nope']:
    a=json.load(open('$OUT/k_'+v+'.json'))
    print(v, round(a['16x16']['us_per_launch'],3), 'tiny', round(a['tiny_kernel_us_per_launch'],3))
" &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.log 2>&1 && tail -1 $OUT/bench_20_5.log | cut -c1-230 &&
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > $OUT/bench_300.log 2>&1 && tail -1 $OUT/bench_300.log | cut -c1-230
