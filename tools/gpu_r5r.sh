#!/bin/bash
# Round 5 session r: the full-schedule R-D pins that have reference runs so far (kodim04 portrait,
# the default decoder once its reference seed exists).  Usage: bash tools/gpu_r5r.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5r}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== rd_full" | tee -a "$OUT/steps.log"
(cd /tmp && timeout -k 10 900 python -u -m pytest -m gpu -x -v -s --timeout 600 --timeout-method thread \
    "$ROOT/tests/test_rd_gpu.py" -k "full_schedule") > "$OUT/rd_full.log" 2>&1
rc=$?
echo "   rc=$rc" | tee -a "$OUT/steps.log"
grep -E "c3x full|passed|failed|skipped" "$OUT/rd_full.log" | cut -c1-300
exit $rc
