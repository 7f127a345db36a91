#!/bin/bash
# A/B of the fused kernel's 1x1 head forms (--head valu / mfma): fused-path parity tests, then
# the quick bench alternating the two.  Usage (GPU box, repo root): bash tools/ab_head.sh OUTDIR
set -u
OUT=${1:-gpurun_out/abhead}
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
Q="--steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 10"
step pytest_fwd 400 python -u -m pytest tests/test_forward.py -m gpu -x -q -k fused --timeout 200 --timeout-method thread
step bench_mfma 300 python bench.py $Q --head mfma
step bench_valu 300 python bench.py $Q --head valu
step bench_mfma2 300 python bench.py $Q --head mfma
step bench_valu2 300 python bench.py $Q --head valu
for f in bench_mfma bench_valu bench_mfma2 bench_valu2; do
  tail -c 3000 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$f', d['value'], d['stage_ms_per_step'], d['roofline']['frac'], d['path_a_1080p']['stage_ms_per_step'])" | tee -a "$OUT/steps.log"
done
