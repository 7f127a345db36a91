#!/bin/bash
# Round-3 A/B session on one GPU box (repo root): parity tests of the changed kernels, then
# the current library against tools/ablib/$1 on the headline path (quick bench, alternating)
# and the training step (tools/bench_train.py), then a kernel trace of the quick bench.
# Usage: bash tools/ab_r3.sh OTHER.so OUTDIR
set -u
OTHER=$(pwd)/tools/ablib/$1
OUT=$(pwd)/${2:-gpurun_out/ab_r3}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_forward.py tests/test_api_mirror.py tests/test_train_gpu.py \
    tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py tests/test_decode_gpu.py -m gpu -x -q --timeout 300 \
    --timeout-method thread
step lat_new 200 python tools/decode_latency.py 2
step lat_other 200 env CCMI_LIB=$OTHER python tools/decode_latency.py 2
Q="--steps 30 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 5 --hd-decode-reps 0"
for i in 1 2; do
    step bench_new_$i 180 python bench.py $Q
    step bench_other_$i 180 env CCMI_LIB=$OTHER python bench.py $Q
    step train_new_$i 200 python tools/bench_train.py 8
    step train_other_$i 200 env CCMI_LIB=$OTHER python tools/bench_train.py 8
done
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $Q
step trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- \
    python3 tools/bench_train.py 8
echo "all steps passed" | tee -a "$OUT/steps.log"
