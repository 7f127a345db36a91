#!/bin/bash
# One GPU session: parity tests, MFMA probe, A/B of the fused-synthesis head and of the
# batched decoder tail.  Every GPU step has its own time limit; the first failure ends it.
# Usage (on the GPU box, from the repo root): bash tools/gpu_check.sh OUTDIR
set -u
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
step() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step mfma_probe 60 ./tools/mfma_probe
QUICK="--steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
step bench_mfma_head 300 python bench.py $QUICK
step bench_valu_head 300 env CCMI_SYN_VALU_HEAD=1 python bench.py $QUICK
step bench_mfma_head_serial 300 python bench.py $QUICK --serial
step ab_tail_batched 600 python tools/ab_decode.py 64
step ab_tail_serial 600 env CCMI_DEC_TAIL_SERIAL=1 python tools/ab_decode.py 64
echo "all steps passed" | tee -a "$OUT/steps.log"
