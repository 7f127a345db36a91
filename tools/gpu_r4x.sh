#!/bin/bash
# Round 4, session x: ReLU mask of the 3x3 backward applied in place by the input-gradient launch (weight-gradient launch reads g_pre, no activation planes) for the
# training ARM kernels and t_head_bwd: training parity tests, then kernel traces and ms per
# iteration (hop ARM 16,2 and the reference default ARM 24,2) against tools/ablib/r4u.so.
# Usage: bash tools/gpu_r4o.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4x}
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
run pytest_train 600 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py tests/test_sanity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  run new$r 200 python tools/bench_train.py 8 --no-cpu
  run r4u_$r 200 python tools/bench_train.py 8 --no-cpu --lib $ROOT/tools/ablib/r4u.so
  run new_arm24_$r 200 python tools/bench_train.py 8 --no-cpu --default-arch
  run r4u_arm24_$r 200 python tools/bench_train.py 8 --no-cpu --default-arch --lib $ROOT/tools/ablib/r4u.so
done
run trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- python3 tools/bench_train.py 8 --no-cpu
run trace_train_r4u 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_r4u -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/r4u.so
run trace_train_arm24 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_arm24 -o run -- python3 tools/bench_train.py 8 --no-cpu --default-arch
run trace_train_arm24_r4u 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_arm24_r4u -o run -- python3 tools/bench_train.py 8 --no-cpu --default-arch --lib tools/ablib/r4u.so
echo "all steps passed" | tee -a "$OUT/steps.log"
