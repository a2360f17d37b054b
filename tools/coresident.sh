#!/bin/bash
# Co-residency of kernels from several processes on one GPU
# (tools/coresident_probe.hip): for each "ranks:blocks:threads:lds" config,
# start that many processes, each launching a kernel whose workgroups wait
# (bounded, 2 s) for every workgroup of every process.  One JSON line per
# process under $OUT/<config>.jsonl.
#   CONFIGS="2:72:768:142168 3:72:768:142168" TAG=r5_cores tools/coresident.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-coresident}
mkdir -p $OUT
cd $ROOT
for c in ${CONFIGS:-2:8:64:1024 3:8:64:1024 2:72:768:142168 3:72:768:142168}; do
  IFS=: read R NB NT LDS <<< "$c"
  d=$(mktemp -d)
  pids=()
  for ((r = 0; r < R; r++)); do
    timeout -k 5 40 ./tools/coresident_probe $r $R $d $NB $NT $LDS 20 > $d/out.$r 2>&1 &
    pids+=($!)
  done
  worst=0
  for p in "${pids[@]}"; do wait $p; rc=$?; [ $rc -gt $worst ] && worst=$rc; done
  cat $d/out.* > $OUT/cfg_${R}_${NB}_${NT}_${LDS}.jsonl
  echo "config $c (worst rc $worst):"; cut -c1-300 $OUT/cfg_${R}_${NB}_${NT}_${LDS}.jsonl
  rm -rf $d
  # a crash or a time limit ends the run (1 = a wait timed out: reported, not fatal)
  [ $worst -le 1 ] || exit $worst
done
echo "== done"
