# Native-runtime throughput across grid sizes and dtypes (one GPU).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
python -m stsphere.ops.build > gpurun_out/build.log 2>&1 || exit 2
: > gpurun_out/size_sweep.log
for v in "--N 96" "--N 96 --dtype fp32" "--N 180" "--N 360 --steps 100 --warmup 10" "--N 720 --steps 40 --warmup 5" "--N 720 --steps 40 --warmup 5 --dtype fp32" "--N 720 --steps 40 --warmup 5 --tiles-per-edge 1"; do
  timeout -k 10 300 python bench.py $v > gpurun_out/sz.log 2>&1 || { tail -5 gpurun_out/sz.log; exit 1; }
  echo "$v :: $(grep '^{' gpurun_out/sz.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), "us/step", "%.3e cell-updates/s" % d["value"])')" | tee -a gpurun_out/size_sweep.log
done
