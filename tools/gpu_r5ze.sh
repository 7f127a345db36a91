#!/bin/bash
# Round 5 session ze: what bounds t_sp_bwd<3> after r5zd -- isolated training traces of the product library
# and the diagnostic variants of tools/spb_diag.sh (NOLOAD / NODW / NODX / NOBORDER; wrong
# results by design, timing only).  Usage: bash tools/gpu_r5ze.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5ze}
mkdir -p "$OUT"
export TMPDIR=/tmp
export CCMI_ARM_OVERLAP=0
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
for v in base noload nodw nodx noborder; do
  if [ $v = base ]; then unset CCMI_LIB; else export CCMI_LIB=$ROOT/tools/ablib/spb_$v.so; fi
  run trace_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$v -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
done
echo "all steps passed" | tee -a "$OUT/steps.log"
