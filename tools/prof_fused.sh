#!/bin/bash
# Where the fused decode kernel spends its time: in-kernel phase stamps (diagnostic build),
# the synthesis micro-benchmark, a kernel trace of the serial bench, and two SQ counter
# passes (each pass its own run, within the per-block slot limits).
# Usage (GPU box, repo root): bash tools/prof_fused.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/prof_fused}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
BENCH="$ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0 --serial"
run stamps 120 env CCMI_LIB=$ROOT/cool-chic_amd/lib/diag/libccmi_stamps.so python3 $ROOT/tools/prof_fused.py
run syn_micro 120 python3 $ROOT/tools/syn_micro.py
run trace 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python3 $BENCH
run pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc1 -- python3 $BENCH
run pmc2 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc2 -- python3 $BENCH
echo "all steps passed" | tee -a "$OUT/steps.log"
