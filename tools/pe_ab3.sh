#!/bin/bash
# Where the no-panel-edge overhead comes from (C96 16x16, same box, graph-timed
# stage launches, panel-edge bits cleared in every variant so only the code
# shape differs): prod vs pe0 (canonical edge layout) vs pnotab (no table
# loads) vs pnoslot (no panel-edge selects in the flux) vs prepe (d318046).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-peab}
mkdir -p $OUT
cd $ROOT
for v in prod pe0 pnotab pnoslot prepe prod_pe; do
  var=$v; flag=--no-pedge
  [ $v = prod ] && var=""
  [ $v = prod_pe ] && { var=""; flag=""; }
  STSP_VARIANT=$var timeout -k 10 200 python -u tools/kprobe.py --blocks 16x16 $flag > $OUT/k_$v.json 2>> $OUT/k.err || exit $?
done
python -c "
import json
for v in ['prod','pe0','pnotab','pnoslot','prepe','prod_pe']:
    a=json.load(open('$OUT/k_'+v+'.json'))
    print(v, round(a['16x16']['us_per_launch'],3), 'tiny', round(a['tiny_kernel_us_per_launch'],3))
"
