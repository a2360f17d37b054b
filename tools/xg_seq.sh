#!/bin/bash
# tools/xg_seq_probe.py for several "ranks:t:K:launch[:N]" configs (shared GPU)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-xg_seq}
mkdir -p $OUT
cd $ROOT
port=29533
for c in ${CONFIGS:-3:2:20:graph}; do
  IFS=: read R T K LA NN <<< "$c"
  NN=${NN:-96}
  port=$((port + 1))
  STSP_SHARE_GPU=1 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node $R \
    --master-addr 127.0.0.1 --master-port $port tools/xg_seq_probe.py --N $NN --t $T --K $K --launch $LA \
    > $OUT/seq_${R}_${T}_${K}_${LA}_$NN.log 2>&1
  rc=$?
  echo "config $c rc=$rc"
  grep '^{' $OUT/seq_${R}_${T}_${K}_${LA}_$NN.log | cut -c1-1500
  [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
done
echo "== done"
