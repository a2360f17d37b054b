#!/bin/bash
# Hand-off protocol A/B on a one-GPU box: the xGMI GPU tests, the loopback probe
# and a 2-rank shared-GPU bench rehearsal, once per library variant
# (VARIANTS, default: "" = the production build, xgt = tagged granules).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; }
for v in ${VARIANTS:-prod xgt}; do
  [ "$v" = prod ] && export STSP_VARIANT= || export STSP_VARIANT=$v
  echo "== variant '$v': pytest xgmi"
  timeout -k 10 400 python -u -m pytest tests/test_xgmi.py -q -x --timeout 120 --timeout-method thread > $OUT/xgt_pytest_$v.log 2>&1
  rc=$?; tail -3 $OUT/xgt_pytest_$v.log
  if fatal $rc || [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
  echo "== variant '$v': loopback probe"
  timeout -k 10 200 python tools/xg_fence_probe.py --N 96 --t 2 >> $OUT/xgt_probe.jsonl 2> $OUT/xgt_probe_$v.err
  rc=$?; tail -1 $OUT/xgt_probe.jsonl
  if [ $rc -ne 0 ]; then echo "probe rc=$rc"; tail -5 $OUT/xgt_probe_$v.err; exit $rc; fi
  for n in ${RANKS:-2}; do
    echo "== variant '$v': bench rehearsal, $n ranks on one GPU"
    STSP_SHARE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 300 --warmup 30 \
        > $OUT/xgt_rehearse_${v}_$n.log 2>&1
    rc=$?; grep -h "^{" $OUT/xgt_rehearse_${v}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"n_gpus\"], d[\"config\"][\"comm\"], 1e3*d[\"ms_per_step\"], \"us/step diff_vs_1gpu\", d[\"max_abs_diff_vs_1gpu\"], d[\"finite\"])"
    if [ $rc -ne 0 ]; then echo "rehearsal rc=$rc"; tail -20 $OUT/xgt_rehearse_${v}_$n.log; exit $rc; fi
  done
done
echo "== done"
