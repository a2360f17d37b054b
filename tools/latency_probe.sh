set -u
cd $GRAFT_REPO_ROOT
python -m stsphere.ops.build --all > gpurun_out/build.log 2>&1 || exit 2
for lim in 1 8 64 216; do
  timeout -k 10 120 python tools/kprobe.py --blocks 16x16 --limit $lim > gpurun_out/kp_$lim.json 2>&1 || exit 3
  echo "limit=$lim $(python3 -c "import json;d=json.load(open('gpurun_out/kp_$lim.json'));print(d['16x16']['us_per_launch'], d['tiny_kernel_us_per_launch'])")"
done
timeout -k 10 120 python tools/kprobe.py --blocks 16x16 --limit 1 --stamps > gpurun_out/kp_1s.json 2>&1 || exit 4
python3 -c "import json;d=json.load(open('gpurun_out/kp_1s.json'));print(d['16x16'])"
