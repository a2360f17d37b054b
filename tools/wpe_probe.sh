#!/bin/bash
# Waves-per-SIMD probe on the streaming grids: graph-timed stage launches of
# the production library (amdgpu_waves_per_eu(5) for the multi-block-per-CU
# shapes) against variants built for 6 and 7 waves per SIMD (fewer VGPRs, more
# spills).  Same box for every row; each run has its own limit.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-wpe}
mkdir -p $OUT
cd $ROOT
for v in prod wpe6 wpe7; do
  var=""; [ $v != prod ] && var=$v
  for dt in fp64 fp32; do
    for N in 720 360; do
      STSP_VARIANT=$var timeout -k 10 200 python -u tools/kprobe.py --N $N --dtype $dt --blocks ${BLOCKS:-16x8,8x8} \
        > $OUT/k_${v}_${dt}_$N.json 2>> $OUT/k.err || exit $?
    done
  done
done
python -c "
import json
for dt in ['fp64','fp32']:
  for N in [720,360]:
    for v in ['prod','wpe6','wpe7']:
      a=json.load(open('$OUT/k_%s_%s_%d.json' % (v, dt, N)))
      print(dt, 'C%d' % N, v, {k: round(x['us_per_launch'],2) for k,x in a.items() if isinstance(x, dict)})
" | tee $OUT/summary.txt
# registers per variant (kernel trace: VGPR / scratch of the 8x8 and 16x8 fp64 bodies)
cd /tmp && export TMPDIR=/tmp
for v in prod wpe6 wpe7; do
  var=""; [ $v != prod ] && var=$v
  STSP_VARIANT=$var timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/kt_$v -o kt --output-format csv -- \
    python3 $ROOT/tools/kprobe.py --N 360 --dtype fp64 --blocks 16x8,8x8 --reps 5 > $OUT/kt_$v.log 2>&1 || exit $?
done
cd $ROOT
python3 - <<PY | tee -a $OUT/summary.txt
import csv, glob
for v in ['prod', 'wpe6', 'wpe7']:
    seen = set()
    for f in glob.glob('$OUT/kt_%s/**/*kernel_trace.csv' % v, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if 'stage_kernel<double' in k and k not in seen:
                seen.add(k)
                print(v, k.split('stage_kernel')[1].split('(')[0], 'vgpr', r.get('Arch_VGPR_Count'), 'accum', r.get('Accum_VGPR_Count'),
                      'sgpr', r.get('SGPR_Count'), 'scratch', r.get('Scratch_Size'), 'lds', r.get('LDS_Block_Size'))
PY
