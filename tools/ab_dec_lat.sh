#!/bin/bash
# Path B A/B: decode parity on the current library, then single-stream latency
# (tools/decode_latency.py) and batch throughput (tools/bench_decode.py) for the current
# library and tools/ablib/$1.  Usage (GPU box, repo root): bash tools/ab_dec_lat.sh OTHER OUTDIR
set -u
OTHER=$(pwd)/tools/ablib/$1
OUT=${2:-gpurun_out/abdec}
mkdir -p "$OUT"
step() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
step pytest_dec 400 python -u -m pytest tests/test_decode_gpu.py tests/test_codec_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread
step lat_new 300 python tools/decode_latency.py 2
step lat_other 300 env CCMI_LIB=$OTHER python tools/decode_latency.py 2
step thr_new 300 python tools/bench_decode.py 16 64
step thr_other 300 env CCMI_LIB=$OTHER python tools/bench_decode.py 16 64
