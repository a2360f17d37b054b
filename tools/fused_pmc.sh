#!/bin/bash
# PMC counters of the fused C96 step (one 100-step launch of bench.py), one
# rocprofv3 --pmc pass per counter set (each set within the per-block limits:
# 8 SQ, 4 TCC with FETCH_SIZE = 3 and WRITE_SIZE = 2), each under a KILL limit.
#   TAG=r5_pmc bash tools/fused_pmc.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-fused_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
           "WRITE_SIZE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc$i -o k --output-format csv -- \
    python3 $ROOT/bench.py --steps 100 --warmup 2 > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; exit 3; }
  i=$((i+1))
done
python3 $ROOT/tools/pmc_summary.py fused_step_kernel $OUT > $OUT/summary.txt
cat $OUT/summary.txt
