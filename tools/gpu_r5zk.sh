#!/bin/bash
# Round 5 session zk: the training step (final round-5 kernels)'s timeline with the ARM on its side stream (kernel trace
# of tools/bench_train.py at the default CCMI_ARM_OVERLAP) and the SQ counters of the training
# kernels, each alone (CCMI_ARM_OVERLAP=0).  Usage: bash tools/gpu_r5zk.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5zk}
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
run step 300 python3 $ROOT/tools/bench_train.py 8 --no-cpu
run trace_ovl 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_ovl -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
export CCMI_ARM_OVERLAP=0
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    run pmc$i 120 rocprofv3 --pmc $grp --kernel-include-regex "t_arm|t_head_bwd|t_sp_bwd|t_sp_fwd|t_head_fwd|t_lvl_bwd" --output-format csv \
        -d $OUT/pmc/p$i -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
done
echo "all steps passed" | tee -a "$OUT/steps.log"
