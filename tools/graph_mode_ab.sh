# STSP_GRAPH_MODE bits: 1 global capture, 2 instantiate-with-flags (STSP_GRAPH_IFLAGS), 4 upload, 8 launch on the null stream
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
python -m stsphere.ops.build > gpurun_out/build.log 2>&1 || exit 2
for f in 1 8 9; do
  echo "iflags $f: $(STSP_GRAPH_MODE=2 STSP_GRAPH_IFLAGS=$f timeout -k 10 120 python tools/runtime_ab.py 2>/dev/null | tail -1 | cut -c1-200)"
done
