cd $GRAFT_REPO_ROOT
python -m stsphere.ops.build --all > gpurun_out/build.log 2>&1 || exit 2
timeout -k 10 200 python tools/persist_probe.py 96 2>&1 | grep -v amdgpu.ids
