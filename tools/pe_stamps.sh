#!/bin/bash
# Same-box phase stamps of the stage kernel (diag library) with and without the
# panel-edge bits, cold and with a warm instruction cache (STSP_DIAG_REPEAT=1:
# the idempotent body runs twice, the stamps keep the second pass).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-pest}
mkdir -p $OUT
cd $ROOT
timeout -k 10 200 python -u tools/kprobe.py --stamps --blocks 16x16 > $OUT/pe.json 2> $OUT/err.txt &&
timeout -k 10 200 python -u tools/kprobe.py --stamps --blocks 16x16 --no-pedge > $OUT/nope.json 2>> $OUT/err.txt &&
STSP_DIAG_REPEAT=1 timeout -k 10 200 python -u tools/kprobe.py --stamps --blocks 16x16 > $OUT/pe_warm.json 2>> $OUT/err.txt &&
STSP_DIAG_REPEAT=1 timeout -k 10 200 python -u tools/kprobe.py --stamps --blocks 16x16 --no-pedge > $OUT/nope_warm.json 2>> $OUT/err.txt
