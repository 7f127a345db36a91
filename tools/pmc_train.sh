#!/bin/bash
# SQ counters of the GPU training kernels (tools/bench_train.py), one rocprofv3 pass per
# counter group.  Usage (GPU box): bash tools/pmc_train.sh TAG [B]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_train_${1:-r2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "t_arm|t_head_bwd|t_sp_bwd|t_head_fwd|t_lvl_bwd" --output-format csv \
        -d "$OUT/p$i" -o run -- python3 "$R/tools/bench_train.py" ${2:-8} --no-cpu > "$OUT/p$i.log" 2>&1
done
echo done
