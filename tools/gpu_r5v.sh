#!/bin/bash
# Round 5 session v: the upsampling levels in XCD-aware order with the channel job fastest
# (balanced per XCD) against tools/ablib/r5v_base.so -- forward + training parity, headline
# A/B interleaved, the pyramid's FETCH.  Usage: bash tools/gpu_r5v.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5v}
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
run tests 600 $PT $ROOT/tests/test_forward.py $ROOT/tests/test_train_gpu.py
Q="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0 --no-single-stream"
for r in 1 2 3; do
  run a_base_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5v_base.so python3 $Q
  run a_new_$r 300 python3 $Q
done
for r in 1 2; do
  run step_base_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5v_base.so python3 $ROOT/tools/bench_train.py 8 --no-cpu
  run step_new_$r 300 python3 $ROOT/tools/bench_train.py 8 --no-cpu
done
run fetch_new 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_new -o run -- python3 $ROOT/tools/pipe_steps.py 32 10 serial
echo "all steps passed" | tee -a "$OUT/steps.log"
