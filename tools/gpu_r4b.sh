#!/bin/bash
# Round 4, session b: training-step A/B (round-3 library vs this round's t_arm16 / t_head_bwd,
# 3- and 4-wave builds of t_arm16), kernel trace of the training bench, and s_memtime stamps of
# the path-B latency kernel on the highest-rate class-B stream.
# Usage (GPU box, repo root): bash tools/gpu_r4b.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
run pytest_train 600 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  run new$r 200 python tools/bench_train.py 8 --no-cpu
  run w4_$r 200 env CCMI_LIB=$ROOT/tools/ablib/w4.so python tools/bench_train.py 8 --no-cpu
  run r3_$r 200 env CCMI_LIB=$ROOT/tools/ablib/r3base.so python tools/bench_train.py 8 --no-cpu
done
run trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- python3 tools/bench_train.py 8 --no-cpu
run trace_train_w4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_w4 -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/w4.so
run trace_train_r3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_r3 -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/r3base.so
run stamps_B 200 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_stamps.so python tools/prof_decode_one.py B-BQTerrace-lmbda-00001_1920x1080_50p_yuv420_8b.cool
run stamps_E 200 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_stamps.so python tools/prof_decode_one.py
echo "all steps passed" | tee -a "$OUT/steps.log"
