#!/bin/bash
# Training-step check on the GPU box (repo root): parity tests, ms per iteration, kernel trace.
# Usage: bash tools/gpu_train_check.sh OUTDIR
set -u
OUT=$(pwd)/${1:-gpurun_out/train_check}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
step pytest_train 400 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py \
    tests/test_codec_e2e.py -m gpu -x -q --timeout 200 --timeout-method thread
step train 200 python tools/bench_train.py 8
step train2 200 python tools/bench_train.py 8
step trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- \
    python3 tools/bench_train.py 8
echo "all steps passed" | tee -a "$OUT/steps.log"
