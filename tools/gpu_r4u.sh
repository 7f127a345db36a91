#!/bin/bash
# Round 4, session u: compile-time taps on the fused kernel's border windows (both parities'
# chains + a select) and wave sums in t_sp_bwd<2>: forward + training parity tests, then the
# headline leg, the training step and kernel traces against tools/ablib/r4p.so.
# Usage: bash tools/gpu_r4u.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4u}
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
run pytest 600 python -u -m pytest tests/test_forward.py tests/test_api_mirror.py tests/test_train_gpu.py tests/test_mirror_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
QB="bench.py --steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
for r in 1 2; do
  run new$r 300 python3 $QB
  run r4p_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r4p.so python3 $QB
  run train_new$r 200 python tools/bench_train.py 8 --no-cpu
done
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $QB
run trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- python3 tools/bench_train.py 8 --no-cpu
export CCMI_LIB=$ROOT/tools/ablib/r4p.so
run trace_r4p 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_r4p -o run -- python3 $QB
echo "all steps passed" | tee -a "$OUT/steps.log"
