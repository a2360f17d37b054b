#!/bin/bash
# Fused-step profile: phase stamps, kernel trace, LDS / VALU counters.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_fprof}
mkdir -p $OUT
cd $ROOT
timeout -k 10 120 python -u tools/fused_probe.py --N ${N:-96} --t ${T:-2} --stamps --stage > $OUT/probe.json 2> $OUT/probe.err || { tail -5 $OUT/probe.err; exit 3; }
cat $OUT/probe.json
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVES" \
           "SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS"; do
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/pmc$i -o k --output-format csv -- \
    python3 $ROOT/tools/fused_probe.py --N ${N:-96} --t ${T:-2} --reps 5 > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; exit 4; }
  i=$((i+1))
done
python3 $ROOT/tools/pmc_summary.py fused_step $OUT
echo "== done"
