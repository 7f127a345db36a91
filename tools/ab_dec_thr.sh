#!/bin/bash
# Path B batch-throughput screen of several libraries (tools/ablib/*.so as arguments) on one GPU
# box: the decode parity tests on the current library, then tools/bench_decode.py (960 class-E
# frames, md5 checked) twice per library, alternating.  Usage: bash tools/ab_dec_thr.sh OUTDIR a.so b.so ...
set -u
OUT=$(pwd)/$1
shift
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_codec_e2e.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
    for l in "$@"; do
        echo "== $l $r"
        timeout -k 10 200 env CCMI_LIB=$(pwd)/tools/ablib/$l python tools/bench_decode.py 16 64 > "$OUT/${l%.so}_$r.log" 2>&1 || { tail -20 "$OUT/${l%.so}_$r.log"; exit 1; }
        tail -n 2 "$OUT/${l%.so}_$r.log" | cut -c1-230
    done
done
echo "all steps passed"
