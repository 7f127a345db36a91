#!/bin/bash
# Round 5 session h: fused kernel with the register / DPP form of the 3x3 layers against the
# library before it (tools/ablib/r5h_base.so): forward parity, then the headline leg three
# times per library, interleaved, the synthesis micro-bench and the phase stamps.
# Usage: bash tools/gpu_r5h.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5h}
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
run fwd_tests 600 $PT $ROOT/tests/test_forward.py $ROOT/tests/test_api_mirror.py
run syn_micro 120 python3 $ROOT/tools/syn_micro.py
run syn_micro_base 120 env CCMI_LIB=$ROOT/tools/ablib/r5h_base.so python3 $ROOT/tools/syn_micro.py
run stamps 120 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_stamps.so python3 $ROOT/tools/prof_fused.py
Q="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0 --no-single-stream"
for r in 1 2 3; do
  run a_base_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5h_base.so python3 $Q
  run a_new_$r 300 python3 $Q
done
run trace 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python3 $Q
echo "all steps passed" | tee -a "$OUT/steps.log"
