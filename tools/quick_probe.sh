#!/bin/bash
# Fast kernel iteration loop on the GPU box: build check, HIP numerics tests,
# kernel probe (graph-timed launch + in-kernel phase stamps), short bench.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
python -m stsphere.ops.build --all > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 2; }
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py tests/test_native_runtime.py ${EXTRA_TESTS:-} -x -q > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_quick.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/kprobe.py --blocks ${BLOCKS:-16x16} ${KPROBE_ARGS:-} > gpurun_out/kprobe.json 2>gpurun_out/kprobe.err || exit $?
timeout -k 10 300 python tools/kprobe.py --stamps --blocks 16x16 ${KPROBE_ARGS:-} > gpurun_out/kprobe_stamps.json 2>>gpurun_out/kprobe.err || exit $?
python -c "import json; a=json.load(open('gpurun_out/kprobe.json')); b=json.load(open('gpurun_out/kprobe_stamps.json')); print({k:v for k,v in a.items() if isinstance(v,dict)}); print(json.dumps(b['16x16'].get('wave_stamp_cycles_median')), b['16x16']['block_cycles_median'])"
timeout -k 10 300 python bench.py --steps 600 --warmup 60 > gpurun_out/bench_quick.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_quick.log | cut -c1-260
if [ "${WARM:-0}" = "1" ]; then
  STSP_DIAG_REPEAT=1 timeout -k 10 300 python tools/kprobe.py --stamps --blocks 16x16 ${KPROBE_ARGS:-} > gpurun_out/kprobe_warm.json 2>>gpurun_out/kprobe.err || exit $?
  python -c "import json; b=json.load(open('gpurun_out/kprobe_warm.json')); print('WARM', json.dumps(b['16x16'].get('wave_stamp_cycles_median')), b['16x16']['block_cycles_median'])"
fi
