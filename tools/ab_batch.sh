#!/bin/bash
# Frames-per-step sweep of the headline leg (path A only).
set -u
OUT=${1:-gpurun_out/abb}
mkdir -p "$OUT"
Q="--steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 0"
for b in ${BATCHES:-8 16 32 8 16}; do
  timeout -k 10 300 python bench.py $Q --batch $b > $OUT/b$b.log 2>&1 || { tail -20 $OUT/b$b.log; exit 1; }
  tail -c 3000 $OUT/b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('B=$b', d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['roofline']['frac'])"
done
