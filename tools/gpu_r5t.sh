#!/bin/bash
# Round 5 session t: XCD-aware tile order for the path-A ARM (tools/ablib/r5t_arm.so) and, on
# top, the upsampling levels (the product build) against tools/ablib/r5t_base.so -- forward +
# training parity, the headline leg interleaved, FETCH / WRITE of every path-A kernel.
# Usage: bash tools/gpu_r5t.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5t}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -1 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run tests 600 $PT $ROOT/tests/test_forward.py $ROOT/tests/test_api_mirror.py $ROOT/tests/test_train_gpu.py
Q="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0 --no-single-stream"
for r in 1 2; do
  run a_base_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5t_base.so python3 $Q
  run a_arm_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5t_arm.so python3 $Q
  run a_new_$r 300 python3 $Q
done
P="$ROOT/tools/pipe_steps.py 32 10 serial"
run fetch_new 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_new -o run -- python3 $P
run write_new 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_new -o run -- python3 $P
export CCMI_LIB=$ROOT/tools/ablib/r5t_base.so
run fetch_base 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_base -o run -- python3 $P
echo "all steps passed" | tee -a "$OUT/steps.log"
