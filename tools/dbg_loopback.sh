cd $GRAFT_REPO_ROOT
python -m stsphere.ops.build --all > gpurun_out/build.log 2>&1 || exit 2
STSP_RT_DEBUG=1 timeout -k 10 300 python -X faulthandler -m pytest tests/test_native_runtime.py -v -x -k "persistent or native_stepper or loopback" > gpurun_out/dbg.log 2>&1
echo rc=$?
grep -v "^  File \"/usr" gpurun_out/dbg.log | head -80
