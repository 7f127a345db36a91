#!/bin/bash
# Occupancy probe of the fused decode kernel: the quick bench with extra dynamic LDS per
# workgroup (2 -> 1 resident workgroups per CU).  Usage (GPU box): bash tools/occ_probe.sh OUT
OUT=${1:-gpurun_out/occ}; mkdir -p $OUT
Q="--steps 30 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 0"
for pad in ${PADS:-0 40000 0 40000}; do
  timeout -k 10 200 env CCMI_SYN_LDS_PAD=$pad python bench.py $Q > $OUT/pad$pad.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$OUT/pad$pad.json').read().strip().splitlines()[-1]); print($pad, d['stage_ms_per_step'])"
done
