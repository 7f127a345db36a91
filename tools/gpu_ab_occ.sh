#!/bin/bash
# A/B vs tools/ablib/prev.so + occupancy probe + fused-kernel FETCH_SIZE pass (GPU box).
set -u
OUT=${1:-gpurun_out/ab_occ}; mkdir -p $OUT
bash tools/ab_lib.sh prev.so $OUT/ab || exit 1
bash tools/occ_probe.sh $OUT/occ || exit 1
Q="$PWD/bench.py --steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex syn_fused --output-format csv -d $OUT/pmc_size -- python3 $Q > $OUT/pmc_size.log 2>&1) || exit 1
echo done
