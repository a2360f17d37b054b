#!/bin/bash
# Multi-rank rehearsal through the bench entry point on a one-GPU box: every
# rank on cuda:0 (STSP_SHARE_GPU=1, gloo group, real IPC between processes).
# Functional check of the paths the driver's 1/2/4/8-GPU scaling run takes;
# the timings are NOT multi-GPU numbers (the ranks share one GPU).  RCCL cannot
# put two ranks on one device, so its path is covered by the loopback tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-rehearsal}
mkdir -p $OUT
cd $ROOT
export STSP_SHARE_GPU=1
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' $OUT/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['config']['comm'], d['config']['parallelism'], 'us/step', round(d['ms_per_step']*1e3,1), 'diff_warm', d['max_abs_diff_vs_1gpu_warmup'], 'diff', d['max_abs_diff_vs_1gpu'], 'graph', d['config']['graph_replayed_steps'], 'eager', d['config']['eager_steps'])" 2>/dev/null)"
  return $rc
}
run g2 --gpus 2 --steps 20 --warmup 5 && \
run g4 --gpus 4 --steps 20 --warmup 5 && \
run g6_t1 --gpus 6 --tiles-per-edge 1 --steps 20 --warmup 5 && \
echo "== done"
# (the 8-rank case is the driver's to run, on a whole node)
