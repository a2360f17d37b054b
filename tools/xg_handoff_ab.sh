#!/bin/bash
# Multi-rank fused step: the in-rank cells by the epoch hand-off or by tagged
# granules (the other ranks' cells through the xGMI ring either way).  The
# loopback share proxies of C96 over 8 GPUs (C36 B=6, C48 B=8), interleaved.
#   TAG=r6_xgh bash tools/xg_handoff_ab.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r6_xgh}
mkdir -p $OUT
cd $ROOT
for cfg in ${CONFIGS:-36:1:6 48:2:8}; do
IFS=: read N T B <<< "$cfg"
for rep in 1 2; do
  for m in epoch tag; do
    tag=C${N}_B${B}_${m}_$rep
    STSP_FUSED_HANDOFF=$m timeout -k 10 180 python -u tools/fused_probe.py --N $N --t $T --B $B --loopback \
      > $OUT/probe_$tag.json 2> $OUT/probe_$tag.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], {k: d.get(k) for k in ('multi20_us_per_step','multi100_us_per_step')})" $OUT/probe_$tag.json $tag
  done
done
done
echo "== xg_handoff_ab done"
