#!/bin/bash
# Round-3 session c (GPU box, repo root): training-step kernel trace, path-B s_memtime
# segment stamps on the highest-rate class-E stream, and the encoder leg at 4 lambdas
# (per-image BD-rate against results.tsv).  Usage: bash tools/gpu_r3c.sh OUTDIR
set -u
OUT=$(pwd)/${1:-gpurun_out/r3c}
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
step pytest_train 300 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread
step train 200 python tools/bench_train.py 8
step trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- \
    python3 tools/bench_train.py 8
[ -n "${STAMPS:-}" ] && step stamps 200 env CCMI_LIB=$(pwd)/cool-chic_amd/lib/libccmi_stamps.so python tools/prof_decode_one.py
# the encoder leg prints one line at its end: a ticker keeps the run visibly alive
( while sleep 50; do date >> "$OUT/tick.log"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
step enc4 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --decode-reps 0 --hd-steps 0 --hd-decode-reps 0 \
    --encode-lambdas 0.02,0.004,0.001,0.0004
echo "all steps passed" | tee -a "$OUT/steps.log"
