#!/bin/bash
# Multi-rank rehearsal of bench.py on ONE card: 2 ranks, gloo (RCCL needs a GPU per rank),
# short legs.  Checks that barriers / collectives / graph capture match across ranks.
# Usage (GPU box, repo root): bash tools/rehearse_dist.sh OUTDIR
set -u
OUT=${1:-gpurun_out/rehearse}
mkdir -p "$OUT"
export CCMI_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --decode-reps 2 \
    --hd-steps 10 --hd-decode-reps 2 --encode-images 2 --encode-scale 0.02 > "$OUT/bench2.log" 2>&1
rc=$?
tail -c 3000 "$OUT/bench2.log"
exit $rc
