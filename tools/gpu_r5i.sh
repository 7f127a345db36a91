#!/bin/bash
# Round 5 session i: t_head_bwd_t with pixel-minor LDS rows (128-bit MFMA operand reads) and
# the fused kernel's head-record prefetch.  Training + forward parity, the training step A/B
# against tools/ablib/r5h_base.so, the decode headline A/B against tools/ablib/r5i_3x3.so,
# the isolated training trace.  Usage: bash tools/gpu_r5i.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5i}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run train_tests 600 $PT $ROOT/tests/test_train_gpu.py $ROOT/tests/test_mirror_train_gpu.py
run fwd_tests 300 $PT $ROOT/tests/test_forward.py
for r in 1 2; do
  run step_base_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5h_base.so python3 $ROOT/tools/bench_train.py 8 --no-cpu
  run step_new_$r 300 python3 $ROOT/tools/bench_train.py 8 --no-cpu
done
Q="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0 --no-single-stream"
for r in 1 2 3; do
  run a_3x3_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5i_3x3.so python3 $Q
  run a_new_$r 300 python3 $Q
done
run stamps 120 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_stamps.so python3 $ROOT/tools/prof_fused.py
export CCMI_ARM_OVERLAP=0
run trace_iso 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_iso -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
echo "all steps passed" | tee -a "$OUT/steps.log"
