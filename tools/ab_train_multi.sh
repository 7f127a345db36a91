#!/bin/bash
# Training-step screen of several libraries (tools/ablib/*.so as arguments, plus the current
# one): tools/bench_train.py 8 twice each, alternating.  Usage: bash tools/ab_train_multi.sh OUTDIR a.so ...
set -u
OUT=$(pwd)/$1
shift
mkdir -p "$OUT"
for r in 1 2; do
    echo "== cur $r"
    timeout -k 10 200 python tools/bench_train.py 8 > "$OUT/cur_$r.log" 2>&1 || exit 1
    tail -1 "$OUT/cur_$r.log"
    for l in "$@"; do
        echo "== $l $r"
        timeout -k 10 200 env CCMI_LIB=$(pwd)/tools/ablib/$l python tools/bench_train.py 8 > "$OUT/${l%.so}_$r.log" 2>&1 || exit 1
        tail -1 "$OUT/${l%.so}_$r.log"
    done
done
echo "all steps passed"
