#!/bin/bash
# Round 5 session f: the R-D parity tests with the round-5 bands (pooled-sigma c3x x0.1 bands,
# 0.15 dB / 4 % full-schedule bands), then the fused kernel's phase breakdown
# (tools/prof_fused.sh: stamps, trace, SQ counters).  Usage: bash tools/gpu_r5f.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5f}
mkdir -p "$OUT"
export TMPDIR=/tmp
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
run rd_tests 900 python -u -m pytest $ROOT/tests/test_rd_gpu.py -m gpu -v -s --timeout 600 --timeout-method thread
cd $ROOT && bash tools/prof_fused.sh ${1:-gpurun_out/r5f}/prof_fused
echo "all steps passed" | tee -a "$OUT/steps.log"
