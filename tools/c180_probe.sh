#!/bin/bash
# C180 (n = 90, 16x8 blocks, partial blocks) stage cost: production with and
# without the panel-edge bits, and the pre-panel-edge library (timing only).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-c180}
mkdir -p $OUT
cd $ROOT
for v in prod nope prepe; do
  var=""; flag=""
  [ $v = nope ] && flag=--no-pedge
  [ $v = prepe ] && var=prepe
  STSP_VARIANT=$var timeout -k 10 200 python -u tools/kprobe.py --N ${N:-180} --blocks ${BLOCKS:-16x8,8x8,16x16} $flag > $OUT/k_$v.json 2>> $OUT/k.err || exit $?
done
python -c "
import json
for v in ['prod','nope','prepe']:
    a=json.load(open('$OUT/k_'+v+'.json'))
    print(v, {k: round(x['us_per_launch'],2) for k,x in a.items() if isinstance(x, dict)})
"
