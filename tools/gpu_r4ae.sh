#!/bin/bash
# Round 4, session ae: the training head forward (t_head_fwd) with the scaled ReLU (clamp on the
# last hidden FMA): training parity tests, ms per iteration and kernel traces against the
# committed training code (tools/ablib/r4y.so).  Usage: bash tools/gpu_r4ae.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4ae}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
run pytest_train 600 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2 3; do
  run new$r 200 python tools/bench_train.py 8 --no-cpu
  run r4y_$r 200 python tools/bench_train.py 8 --no-cpu --lib $ROOT/tools/ablib/r4y.so
done
run trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- python3 tools/bench_train.py 8 --no-cpu
run trace_train_r4y 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_r4y -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/r4y.so
echo "all steps passed" | tee -a "$OUT/steps.log"
