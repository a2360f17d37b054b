#!/bin/bash
# IPC copy transport check: the runtime / IPC GPU tests, the one-process
# transport probe, then the 2-rank shared-GPU IPC bench row.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-ipc_k}
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_native_runtime.py tests/test_solver_gpu.py -k "ipc or native" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for f in 0 1; do
  STSP_IPC_FORK=$f timeout -k 10 200 python -u tools/transport_probe.py > $OUT/transport_probe_fork$f.json 2> $OUT/transport_probe.err || { tail -20 $OUT/transport_probe.err; exit 1; }
  echo "fork=$f"; cat $OUT/transport_probe_fork$f.json
done
STSP_SHARE_GPU=1 timeout -k 10 240 python -u bench.py --gpus 2 --N 96 --tiles-per-edge 2 --steps 20 --warmup 5 \
  --runtime native --comm ipc --timeout 240 > $OUT/ipc_row.log 2>&1 || { tail -20 $OUT/ipc_row.log; exit 1; }
grep -E "^\{" $OUT/ipc_row.log | cut -c1-400
STSP_IPC_FORK=1 STSP_SHARE_GPU=1 timeout -k 10 240 python -u bench.py --gpus 2 --N 96 --tiles-per-edge 2 --steps 20 --warmup 5 \
  --runtime native --comm ipc --timeout 240 > $OUT/ipc_row_fork1.log 2>&1 || { tail -20 $OUT/ipc_row_fork1.log; exit 1; }
grep -E "^\{" $OUT/ipc_row_fork1.log | cut -c1-400
echo "== all done"
