#!/bin/bash
# Path B latency screen of several libraries (tools/ablib/*.so given as arguments, plus the
# current one) on one GPU box: tools/decode_latency.py (md5 checked per stream) twice each,
# alternating.  Usage: bash tools/ab_dec_multi.sh OUTDIR lib1.so lib2.so ...
set -u
OUT=$(pwd)/$1
shift
mkdir -p "$OUT"
for r in 1 2; do
    echo "== cur $r"
    timeout -k 10 200 python tools/decode_latency.py 2 > "$OUT/cur_$r.log" 2>&1 || exit 1
    tail -1 "$OUT/cur_$r.log" | cut -c1-120
    for l in "$@"; do
        echo "== $l $r"
        timeout -k 10 200 env CCMI_LIB=$(pwd)/tools/ablib/$l python tools/decode_latency.py 2 > "$OUT/${l%.so}_$r.log" 2>&1 || exit 1
        tail -1 "$OUT/${l%.so}_$r.log" | cut -c1-120
    done
done
echo "all steps passed"
