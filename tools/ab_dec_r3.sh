#!/bin/bash
# Path B A/B on one GPU box (repo root): decode parity tests, then ccmi_decode_file latency on
# the 15 class-E streams and the 960-stream batch for the current library and tools/ablib/$1,
# alternating.  Usage: bash tools/ab_dec_r3.sh OTHER.so OUTDIR
set -u
OTHER=$(pwd)/tools/ablib/$1
OUT=$(pwd)/${2:-gpurun_out/abdec_r3}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -1 "$OUT/$name.log" | cut -c1-200
    if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
step pytest_dec 400 python -u -m pytest tests/test_decode_gpu.py tests/test_codec_e2e.py tests/test_encode.py -m gpu -x -q \
    --timeout 300 --timeout-method thread
for i in 1 2; do
    step lat_new_$i 200 python tools/decode_latency.py 2
    step lat_other_$i 200 env CCMI_LIB=$OTHER python tools/decode_latency.py 2
done
step thr_new 300 python tools/bench_decode.py 16 64
step thr_other 300 env CCMI_LIB=$OTHER python tools/bench_decode.py 16 64
[ -n "${STAMPS:-}" ] && step stamps 200 env CCMI_LIB=$(pwd)/cool-chic_amd/lib/libccmi_stamps.so python tools/prof_decode_one.py
echo "all steps passed" | tee -a "$OUT/steps.log"
