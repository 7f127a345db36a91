#!/bin/bash
# Round 5 session g: path-A ARM A/B -- bias + residual folded into the accumulator init (the
# default build) and the op_sel weight broadcast (tools/ablib/armopsel.so) against the library
# before both (tools/ablib/r5_prefold.so): forward parity tests on the two new builds, then the
# headline leg three times per library, interleaved.  Usage: bash tools/gpu_r5g.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5g}
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
run fwd_tests 600 $PT $ROOT/tests/test_forward.py $ROOT/tests/test_api_mirror.py $ROOT/tests/test_quantize_gpu.py
run fwd_tests_opsel 600 env CCMI_LIB=$ROOT/tools/ablib/armopsel.so $PT $ROOT/tests/test_forward.py -k "not generic"
Q="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0 --no-single-stream"
for r in 1 2 3; do
  run a_prefold_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5_prefold.so python3 $Q
  run a_fold_$r 300 python3 $Q
  run a_opsel_$r 300 env CCMI_LIB=$ROOT/tools/ablib/armopsel.so python3 $Q
done
echo "all steps passed" | tee -a "$OUT/steps.log"
