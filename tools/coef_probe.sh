#!/bin/bash
# Does the border-slot edge order cost through its scattered edge-coefficient
# loads?  Stage launch time (C96 fp64 16x16, graph-timed) of production vs the
# pcoef probe (coefficients loaded in canonical edge order: timing only).
# Historical: the STSP_PROBE_COEF macro and the pcoef build variant were removed
# after the probe lost (profiles/r2_pe/README.md, v4); re-add them to rerun.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-pcoef}
mkdir -p $OUT
cd $ROOT
for r in 1 2 3; do
  for v in prod pcoef; do
    var=""; [ $v != prod ] && var=$v
    STSP_VARIANT=$var timeout -k 10 120 python -u tools/kprobe.py --N 96 --blocks 16x16 > $OUT/k_${v}_$r.json 2>>$OUT/k.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/k_${v}_$r.json')); print('$v', round(d['16x16']['us_per_launch'],3))" | tee -a $OUT/summary.txt
  done
done
