#!/bin/bash
# Memory-side counters of one stage at a large grid (default C720), one
# rocprofv3 --pmc pass per set (TCC: FETCH_SIZE uses 3, WRITE_SIZE 2 of 4).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
ARGS=${KPROBE_ARGS:---N 720 --dtype fp32}
timeout -k 10 200 python tools/kprobe.py --blocks ${BLOCK:-16x16} $ARGS > gpurun_out/big_kprobe.json 2>gpurun_out/big_kprobe.err || exit $?
cat gpurun_out/big_kprobe.json
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" \
           "WRITE_SIZE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"; do
  timeout -s KILL 90 rocprofv3 --pmc $set -d $ROOT/gpurun_out/big/pmc$i -o k --output-format csv -- python3 $ROOT/tools/kprobe.py --blocks ${BLOCK:-16x16} --reps 10 $ARGS > $ROOT/gpurun_out/big_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $ROOT/gpurun_out/big_$i.log; exit 3; }
  i=$((i+1))
done
python3 $ROOT/tools/pmc_summary.py stage_kernel $ROOT/gpurun_out/big
