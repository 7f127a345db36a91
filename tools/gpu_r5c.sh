#!/bin/bash
# Round 5 session c: the chain kernel with its helper wave (preG chunks off the chain) -- decoder parity tests,
# single-stream latency (class E, class B) against the round-4 library (tools/ablib/r4final.so),
# the stamps build on BQTerrace / FourPeople lambda 1e-4, batch throughput.
# Usage (GPU box, repo root): bash tools/gpu_r5b.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5c}
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD=$ROOT/tools/ablib/r4final.so
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run dec_tests 600 $PT $ROOT/tests/test_decode_gpu.py $ROOT/tests/test_codec_e2e.py $ROOT/tests/test_encode.py
for s in B-BQTerrace-lmbda-00001_1920x1080_50p_yuv420_8b.cool E-FourPeople-lmbda-00001_1280x720_60p_yuv420_8b.cool; do
  run stamps_${s%%_*} 300 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_stamps.so python $ROOT/tools/prof_decode_one.py $s
done
run lat_E_new 300 python $ROOT/tools/decode_latency.py 2
run lat_E_old 300 env CCMI_LIB=$OLD python $ROOT/tools/decode_latency.py 2
run lat_B_new 300 python $ROOT/tools/decode_latency.py 2 'B-*.cool'
run thr_new 300 python $ROOT/tools/bench_decode.py 64
echo "all steps passed" | tee -a "$OUT/steps.log"
