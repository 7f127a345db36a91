#!/bin/bash
# Round 4, session ah: the training ARM on a side stream (CCMI_ARM_OVERLAP = k: at most k
# workgroups per CU, concurrent with the synthesis / upsampling chain), k = 1, 2, 3, against the
# default single-stream build: training parity tests on each, ms per iteration, kernel traces.
# Usage: bash tools/gpu_r4ah.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4ah}
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
for v in 1 2; do
  run pytest_ov$v 600 env CCMI_LIB=$ROOT/tools/ablib/ov$v.so python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
done
for r in 1 2; do
  run base$r 200 python tools/bench_train.py 8 --no-cpu
  for v in 1 2 3; do run ov${v}_$r 200 python tools/bench_train.py 8 --no-cpu --lib $ROOT/tools/ablib/ov$v.so; done
done
run trace_base 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_base -o run -- python3 tools/bench_train.py 8 --no-cpu
run trace_ov2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ov2 -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/ov2.so
echo "all steps passed" | tee -a "$OUT/steps.log"
