#!/bin/bash
# Eager path-A step with the ARM on a second stream concurrent with the decode tail vs one
# stream (GPU box).  Usage: bash tools/ovl_probe.sh OUT
OUT=${1:-gpurun_out/ovl}; mkdir -p $OUT
Q="--steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 0 --no-graph"
for v in serial overlap serial overlap; do
  F=""; [ $v = overlap ] && F="--overlap"
  timeout -k 10 200 python bench.py $Q $F > $OUT/$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done
