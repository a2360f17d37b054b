#!/bin/bash
# Roofline counters of the production stage kernel: HBM bytes (TCC FETCH /
# WRITE_SIZE), VALU instruction mix (fp64 / fp32 FMA, ADD, MUL, TRANS), busy
# cycles.  One rocprofv3 --pmc pass per counter set, each under its own KILL limit.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-roof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run_case() {  # name, kprobe args
  local name=$1; shift
  timeout -k 10 200 python3 $ROOT/tools/kprobe.py "$@" > $OUT/${name}_kprobe.json 2> $OUT/${name}_kprobe.err || return $?
  local i=0
  for set in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
             "WRITE_SIZE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32"; do
    timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/$name/pmc$i -o k --output-format csv -- \
      python3 $ROOT/tools/kprobe.py --reps 10 "$@" > $OUT/${name}_pmc$i.log 2>&1 || { echo "$name pmc $i failed"; tail -3 $OUT/${name}_pmc$i.log; return 3; }
    i=$((i+1))
  done
  python3 $ROOT/tools/pmc_summary.py ${KERNEL:-stage_kernel} $OUT/$name > $OUT/${name}_summary.txt
  echo "== $name"; cat $OUT/${name}_summary.txt
}
# CASES="name:kprobe args;..." (default: the block kernel at C720 fp64 / fp32 and C96);
# KERNEL: the kernel-name substring pmc_summary.py aggregates (march_kernel for 64xR)
IFS=';' read -ra cases <<< "${CASES:-c720_fp64_8x8:--N 720 --dtype fp64 --blocks 8x8;c720_fp32_16x8:--N 720 --dtype fp32 --blocks 16x8;c96_fp64_16x16:--N 96 --dtype fp64 --blocks 16x16}"
for c in "${cases[@]}"; do
  run_case ${c%%:*} ${c#*:} || exit $?
done
