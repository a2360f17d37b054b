set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -m stsphere.ops.build --all > gpurun_out/build.log 2>&1 || exit 2
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 300 python tools/kprobe.py ${KPROBE_ARGS:-} > gpurun_out/kprobe.json 2>gpurun_out/kprobe.err || exit $?
timeout -k 10 300 python tools/kprobe.py --stamps --blocks 16x16 ${KPROBE_ARGS:-} > gpurun_out/kprobe_stamps.json 2>>gpurun_out/kprobe.err || exit $?
cat gpurun_out/kprobe.json gpurun_out/kprobe_stamps.json
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM" \
           "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TD_TD_BUSY TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  timeout -k 10 200 rocprofv3 --pmc $set -d $GRAFT_REPO_ROOT/gpurun_out/pmc$i -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kprobe.py --blocks 16x16 --reps 20 ${KPROBE_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/pmc$i.log 2>&1 || { echo "pmc $i failed"; exit 3; }
  i=$((i+1))
done
echo pmc done
