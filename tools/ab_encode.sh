#!/bin/bash
# Images-per-GPU sweep of the encoder-overfit leg at a fraction of the c3x schedule.
set -u
OUT=${1:-gpurun_out/abe}
SCALE=${2:-0.1}
mkdir -p "$OUT"
Q="--steps 10 --warmup 2 --no-cpu-baseline --decode-reps 0 --hd-decode-reps 0 --hd-steps 0 --batch 8 --encode-scale $SCALE"
for n in 8 16 32; do
  timeout -k 10 400 python bench.py $Q --encode-images $n > $OUT/e$n.log 2>&1 || { tail -20 $OUT/e$n.log; exit 1; }
  tail -c 3000 $OUT/e$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['encoder_overfit']; print('images=$n', e['value'], e['seconds'], e['psnr_db_mean'], e['rate_bpp_mean'])"
done
