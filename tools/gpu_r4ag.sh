#!/bin/bash
# Round 4, session ag: the path-A ARM with the scaled ReLU (clamp on the residual add; inputs, biases and output weights rescaled by powers of two)
# forward parity tests, then the headline leg and kernel traces
# against the committed library (tools/ablib/r4af.so).  Usage: bash tools/gpu_r4ag.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4ag}
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
run pytest 600 python -u -m pytest tests/test_forward.py tests/test_api_mirror.py tests/test_sanity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
QB="bench.py --steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
for r in 1 2 3; do
  run new$r 300 python3 $QB
  run r4af_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r4af.so python3 $QB
done
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $QB
export CCMI_LIB=$ROOT/tools/ablib/r4af.so
run trace_r4af 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_r4af -o run -- python3 $QB
echo "all steps passed" | tee -a "$OUT/steps.log"
