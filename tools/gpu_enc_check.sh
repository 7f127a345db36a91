#!/bin/bash
# Encoder-side GPU checks: training / mirror / quantize tests, then the c3x R-D tests.
# Usage (GPU box, repo root): bash tools/gpu_enc_check.sh OUTDIR [pytest -k expr]
set -u
OUT=${1:-gpurun_out/enc}
K=${2:-}
mkdir -p "$OUT"
step() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
step train 600 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step rd 900 python -u -m pytest tests/test_rd_gpu.py -m gpu -x -q -s -k "${K:-c3x}" --timeout 800 --timeout-method thread
