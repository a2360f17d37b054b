#!/bin/bash
# End-to-end CLI run of the C48 GPU config (BASELINE config 2: 15 days of TC5,
# history, checkpoints, metrics, watchdog, zarr geometry / IC stages, plots),
# then bench.py at the same grid for the steady-state comparison.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-c48run}
mkdir -p $OUT
export PYTHONPATH=$ROOT
CFG=$ROOT/sharding-the-sphere-fall-2025-jax-devlab-examples_amd/configs/c48_1gpu.yaml
cd $OUT
timeout -k 10 400 python -u -m stsphere run $CFG --plot > run.log 2>&1 || { tail -20 run.log; exit 1; }
tail -4 run.log
# second start: geometry and IC are read back from the zarr stages written by the first
timeout -k 10 200 python -u -m stsphere run $CFG --days 1 > run_restart_from_zarr.log 2>&1 || { tail -20 run_restart_from_zarr.log; exit 1; }
tail -2 run_restart_from_zarr.log
cd $ROOT
timeout -k 10 120 python -u bench.py --N 48 --steps 300 --warmup 30 > $OUT/bench_c48.log 2>&1 || { tail -5 $OUT/bench_c48.log; exit 1; }
tail -1 $OUT/bench_c48.log
rm -rf $OUT/run_c48/checkpoints
