#!/bin/bash
# xGMI direct-halo checks on a one-GPU box: GPU tests, then multi-rank bench
# rehearsals with every rank sharing cuda:0 (functional only, not a benchmark).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; }
python -m stsphere.ops.build > $OUT/build.log 2>&1 || { echo build failed; cat $OUT/build.log; exit 2; }
echo "== pytest xgmi"
timeout -k 10 600 python -m pytest tests/test_xgmi.py -q -x > $OUT/xgmi.log 2>&1
rc=$?; tail -5 $OUT/xgmi.log
if fatal $rc; then exit $rc; fi
for n in ${RANKS:-2 4 8}; do
  echo "== bench rehearsal, $n ranks on one GPU"
  STSP_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 30 --warmup 5 \
      ${BENCH_ARGS:-} > $OUT/rehearse_$n.log 2>&1
  rc=$?; grep -h "^{" $OUT/rehearse_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"n_gpus\"], d[\"config\"][\"comm\"], d[\"ms_per_step\"], \"diff_vs_1gpu\", d[\"max_abs_diff_vs_1gpu\"], d[\"finite\"])"; grep -h "\[bench\]" $OUT/rehearse_$n.log | head -5
  if [ $rc -ne 0 ]; then echo "rehearsal rc=$rc"; tail -20 $OUT/rehearse_$n.log; exit $rc; fi
done
echo "== done"
