#!/bin/bash
# Round 4, session l: persistent-grid sizes of t_arm16 (CCMI_AB_ARM_WG, workgroups for the
# batch) and t_head_bwd (CCMI_AB_HEAD_WG): kernel traces of tools/bench_train.py 8 per setting.
# Usage: bash tools/gpu_r4l.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4l}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CFGS:-"2048 1024" "1024 1024" "3072 1024" "4096 1024" "2048 512" "2048 2048" "2048 1024"}; do
    set -- ${cfg/_/ }
    name=arm$1_head$2_$RANDOM
    echo "== $name" | tee -a "$OUT/steps.log"
    CCMI_AB_ARM_WG=$1 CCMI_AB_HEAD_WG=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 tools/bench_train.py 8 --no-cpu > "$OUT/$name.log" 2>&1
    rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
done
echo "all steps passed" | tee -a "$OUT/steps.log"
