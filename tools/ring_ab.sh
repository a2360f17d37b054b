#!/bin/bash
# Ring-layout A/B on one GPU (verdict r5 weak #3): the share proxies of C96
# over 8 GPUs (C36 t=1 B=6 and C48 t=2 B=8: 216 resident blocks each, as in
# profiles/r5_rehearse), in-launch and in loopback (every other tile's window
# cells through the rank's own xGMI ring), with the word-major ring (default
# build) and the round-5 record-major ring (STSP_VARIANT=xgaos), interleaved;
# then one PMC pass per layout counting the write requests to memory.
#   TAG=r6_ring bash tools/ring_ab.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r6_ring}
mkdir -p $OUT
cd $ROOT
for cfg in ${CONFIGS:-36:1:6 48:2:8}; do
IFS=: read N T B <<< "$cfg"
P="--N $N --t $T --B $B"
for rep in 1 2; do
  for v in prod xgaos; do
    for lb in "" "--loopback"; do
      [ "$v" = xgaos ] && [ -z "$lb" ] && continue
      tag=C${N}_B${B}_${v}${lb:+_loopback}_$rep
      STSP_VARIANT=$([ $v = prod ] && echo "" || echo $v) timeout -k 10 180 python -u tools/fused_probe.py $P $lb \
        > $OUT/probe_$tag.json 2> $OUT/probe_$tag.err || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], {k: d.get(k) for k in ('multi20_us_per_step','multi100_us_per_step','graph_us_per_step')})" $OUT/probe_$tag.json $tag
    done
  done
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -o "TCC_EA0_WR[A-Z0-9_]*" $OUT/counters.txt | sort -u > $OUT/wr_counters.txt
cat $OUT/wr_counters.txt | head -20
for v in prod xgaos; do
  export STSP_VARIANT=$([ $v = prod ] && echo "" || echo $v)
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace --stats -d $OUT/pmc_$v -o pmc \
    -- python -u $ROOT/tools/fused_probe.py --N 36 --t 1 --B 6 --loopback --reps 5 > $OUT/pmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
done
echo "== ring_ab done"
