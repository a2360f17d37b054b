set -o pipefail
OUT=gpurun_out/r3_mprobe; mkdir -p $OUT
for v in "" mprobe; do
  for dt in fp64 fp32; do
    for b in 64x4 64x8; do
      STSP_VARIANT=$v timeout -k 10 200 python -u bench.py --runtime native --N 720 --tiles-per-edge 1 --steps 10 --warmup 2 --dtype $dt --block $b > $OUT/b.log 2>&1 || { tail -3 $OUT/b.log; exit 4; }
      echo "variant=$v $dt $b :: $(tail -n 1 $OUT/b.log | cut -c1-140)" | tee -a $OUT/sizes.log
    done
  done
done
