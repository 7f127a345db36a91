#!/bin/bash
# Round 5 session zh: the R-D tests against the merged reference seeds (kodim01 c3x x0.1 seeds 0-3,
# kodim04 full-schedule seeds 0-1) on the current training kernels.  Usage: bash tools/gpu_r5zh.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5zh}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 600 --timeout-method thread $ROOT/tests/test_rd_gpu.py > "$OUT/rd_tests.log" 2>&1
rc=$?
tail -3 "$OUT/rd_tests.log"
exit $rc
