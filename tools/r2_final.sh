#!/bin/bash
# Round-end validation of the tree: GPU tests, driver-style bench, kernel
# stats, smoke(), and the 2/4/6-rank shared-GPU rehearsals through bench.py.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
TAG=${TAG:-r2_final} bash tools/r2_check.sh && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r2_final}/smoke.log 2>&1 && \
tail -1 gpurun_out/${TAG:-r2_final}/smoke.log && \
TAG=${TAG:-r2_final}/rehearsal bash tools/r2_rehearsal.sh
