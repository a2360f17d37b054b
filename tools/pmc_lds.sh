#!/bin/bash
# LDS / VALU counters of the stage kernel (one rocprofv3 --pmc pass per set).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT && mkdir -p gpurun_out
python -m stsphere.ops.build > gpurun_out/build.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"; do
  timeout -k 10 200 rocprofv3 --pmc $set -d $ROOT/gpurun_out/lds/pmc$i -o k --output-format csv -- python3 $ROOT/tools/kprobe.py --blocks 16x16 --reps 20 ${KPROBE_ARGS:-} > $ROOT/gpurun_out/lds_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $ROOT/gpurun_out/lds_$i.log; exit 3; }
  i=$((i+1))
done
python3 $ROOT/tools/pmc_summary.py stage_kernel $ROOT/gpurun_out/lds
