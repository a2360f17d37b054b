#!/bin/bash
# Per-rank share proxies of the multi-GPU C96 run on one GPU (tools/fused_probe.py):
# a rank of an R-GPU run holds 24/R tiles of 48 cells, i.e. the block size the
# residency-aware choice gives it (8 GPUs: 108 blocks of 8; 4: 96 blocks of 12;
# 2: 108 blocks of 16).  One GPU runs a grid whose blocks have that size and are
# all resident (C48 t=2: 216 blocks of 8; C72 t=3: 216 of 12; C96 t=2: 216 of
# 16), once with the in-launch hand-off and once in loopback (every other tile's
# window cells through the rank's own xGMI ring: the multi-GPU protocol).
#   CONFIGS="48:2:8 72:3:12 96:2:16" TAG=r4_share tools/fused_share.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-fused_share}
mkdir -p $OUT
cd $ROOT
for c in ${CONFIGS:-48:2:8 72:3:12 96:2:16}; do
  IFS=: read N T B <<< "$c"
  for lb in "" "--loopback"; do
    tag=C${N}_t${T}_B${B}${lb:+_loopback}
    timeout -k 10 180 python -u tools/fused_probe.py --N $N --t $T --B $B $lb ${PROBE_ARGS:---stamps} \
      > $OUT/probe_$tag.json 2> $OUT/probe_$tag.err || exit $?
    python - "$OUT/probe_$tag.json" "$tag" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["blocks", "graph_us_per_step", "multi20_us_per_step", "multi100_us_per_step", "host_timed_20_us_per_step"]
print(sys.argv[2], {k: d.get(k) for k in keys})
EOF
  done
done
echo "== done"
