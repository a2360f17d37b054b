#!/bin/bash
# Latency of one fused stage with the block count a rank has at C96 / t=2 on
# 2, 4 and 8 GPUs (12, 6, 3 tiles of 48^2), per block shape (kprobe --limit).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/small_grid
mkdir -p $OUT
cd $ROOT
for tiles in 12 6 3; do
  for bs in 16x16 16x8 8x8; do
    bx=${bs%x*}; by=${bs#*x}
    nb=$(( tiles * (48/bx) * (48/by) ))
    timeout -k 10 120 python tools/kprobe.py --blocks $bs --limit $nb > $OUT/t${tiles}_${bs}.json 2>$OUT/err.log || exit $?
    echo "tiles=$tiles $bs blocks=$nb $(python -c "import json;d=json.load(open('$OUT/t${tiles}_${bs}.json'));print(round(d['$bs']['us_per_launch'],3))")"
  done
done
