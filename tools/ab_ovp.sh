#!/bin/bash
# Headline leg: one stream vs ARM concurrent with the upsampling pyramid (--overlap-pyramid).
set -u
OUT=${1:-gpurun_out/abo}
mkdir -p "$OUT"
Q="--steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 0"
for v in serial ovp serial2 ovp2; do
  f=""; case $v in ovp*) f="--overlap-pyramid";; esac
  timeout -k 10 300 python bench.py $Q $f > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  tail -c 3000 $OUT/$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['launch'], d['graph_outputs_equal_eager'], d['eager'], d['stage_ms_per_step'], d['roofline']['frac'])"
done
