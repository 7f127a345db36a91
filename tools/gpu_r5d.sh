#!/bin/bash
# Round 5 session d: tiled t_head_bwd (t_head_bwd_t) -- training parity tests, the 8-frame
# 512x768 step against the round-4 library (tools/ablib/r4final.so), the kernel trace of the
# step (profiles/r5d_train_kernel_stats.csv) and the SQ counters of the training kernels.
# Usage (GPU box, repo root): bash tools/gpu_r5d.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5d}
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
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run dec_tests 600 $PT $ROOT/tests/test_decode_gpu.py
run lat_E 300 python $ROOT/tools/decode_latency.py 2
run train_tests 600 $PT $ROOT/tests/test_train_gpu.py $ROOT/tests/test_mirror_train_gpu.py
run step_new 300 python $ROOT/tools/bench_train.py 8 --no-cpu
run step_old 300 python $ROOT/tools/bench_train.py 8 --no-cpu --lib tools/ablib/r4final.so
run step_new2 300 python $ROOT/tools/bench_train.py 8 --no-cpu
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    run pmc$i 120 rocprofv3 --pmc $grp --kernel-include-regex "t_arm|t_head_bwd|t_sp_bwd|t_head_fwd" --output-format csv \
        -d $OUT/pmc/p$i -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
done
echo "all steps passed" | tee -a "$OUT/steps.log"
