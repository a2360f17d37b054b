#!/bin/bash
# Round-3 final validation on one GPU: whole GPU suite, smoke, the driver-style
# bench (20/5 twice) and 300/30, the size rows (C180 fused, C720 fp64/fp32 with
# the streaming stage and with the block kernel), rocprofv3 kernel stats of the
# 20/5 bench and of C720, PMC passes of the streaming stage at C720.  Every GPU
# step has its own limit; the script stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-r3_final}
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 3; }
grep smoke $OUT/smoke.log
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_20_5_$r.log 2>&1 || exit $?
  tail -n 1 $OUT/bench_20_5_$r.log | cut -c1-200; echo
done
timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 > $OUT/bench_300_30.log 2>&1 || exit $?
tail -n 1 $OUT/bench_300_30.log | cut -c1-200; echo
row() {
  timeout -k 10 240 python -u bench.py "$@" > $OUT/sz.log 2>&1 || { tail -5 $OUT/sz.log; exit 4; }
  echo "$* :: $(tail -n 1 $OUT/sz.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["ms_per_step"]*1e3,2), "us/step", "%.3e" % d["value"], c["runtime"], c["block"])')" | tee -a $OUT/sizes.log
}
row --N 180 --steps 20 --warmup 5
row --N 180 --tiles-per-edge 3 --steps 20 --warmup 5
row --N 720 --tiles-per-edge 1 --steps 10 --warmup 2
row --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype fp32
row --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --block 8x8
row --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype fp32 --block 16x8
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- \
  python3 $ROOT/bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof720 -o bench --output-format csv -- \
  python3 $ROOT/bench.py --N 720 --tiles-per-edge 1 --steps 6 --warmup 2 > $OUT/prof720.log 2>&1 || exit $?
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
           "WRITE_SIZE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32"; do
  for dt in fp64 fp32; do
    timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/pmc_$dt/pmc$i -o k --output-format csv -- \
      python3 $ROOT/tools/kprobe.py --reps 10 --N 720 --t 1 --dtype $dt --blocks 64x4 > $OUT/pmc_${dt}_$i.log 2>&1 || { echo "pmc $dt $i failed"; tail -3 $OUT/pmc_${dt}_$i.log; exit 5; }
  done
  i=$((i+1))
done
for dt in fp64 fp32; do
  timeout -k 10 100 python3 $ROOT/tools/kprobe.py --reps 50 --N 720 --t 1 --dtype $dt --blocks 64x4,64x8,8x8,16x8 > $OUT/kprobe_$dt.json 2>&1
  python3 $ROOT/tools/pmc_summary.py march_kernel $OUT/pmc_$dt > $OUT/pmc_${dt}_summary.txt
  echo "== $dt"; cat $OUT/pmc_${dt}_summary.txt
done
echo "== done"
