set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in "--steps-per-graph 30" "--steps-per-graph 150" "--steps-per-graph 300" "--runtime graph --steps-per-graph 30" "--runtime graph --steps-per-graph 300"; do
  timeout -k 10 200 python bench.py --steps 600 --warmup 60 $v > gpurun_out/bv.log 2>&1 || { tail -5 gpurun_out/bv.log; exit 1; }
  echo "$v :: $(grep '^{' gpurun_out/bv.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,2), "us/step", "%.3e" % d["value"])')"
done
