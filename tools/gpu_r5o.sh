#!/bin/bash
# Round 5 session o: the share of the gradient flush (one atomic per value per workgroup) in
# t_arm16 / t_head_bwd_t -- isolated training traces with the real library and with the
# CCMI_DIAG_NOFLUSH build (flush skipped, wrong results by design).
# Usage: bash tools/gpu_r5o.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5o}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
export CCMI_ARM_OVERLAP=0
run trace_real 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_real -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
export CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_diag_noflush.so
run trace_noflush 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_noflush -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
echo "all steps passed" | tee -a "$OUT/steps.log"
