#!/bin/bash
# PMC passes (one rocprofv3 --pmc set per run) of the pipelined march and of
# the one-stage streaming kernel at C720, fp64 and fp32 (tools/march3_probe.py)
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/m3d; mkdir -p $O
for d in fp64 fp32; do
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" "FETCH_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/$d/pmc$i -o k --output-format csv -- python3 $R/tools/march3_probe.py --N 720 --dtype $d --reps 3 > $O/${d}_pmc$i.log 2>&1 || { echo "pmc $d $i failed"; tail -5 $O/${d}_pmc$i.log; exit 4; }
  i=$((i+1))
done
python3 $R/tools/pmc_summary.py march3_kernel $O/$d > $O/${d}_march3.txt
python3 $R/tools/pmc_summary.py march_kernel $O/$d > $O/${d}_march1.txt
echo "== $d march3"; cat $O/${d}_march3.txt; echo "== $d march (one stage)"; cat $O/${d}_march1.txt
done
