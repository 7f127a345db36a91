#!/bin/bash
# Fused-kernel diagnostics (GPU box): bench with the MFMA head, the VALU head, the no-load
# diagnostic build, and the per-phase stamps.  Usage: bash tools/diag_fused.sh OUTDIR
set -eu
OUT=${1:-gpurun_out/diag}
mkdir -p "$OUT"
Q="--steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
timeout -k 10 300 python bench.py $Q > "$OUT/mfma.json"
timeout -k 10 300 env CCMI_SYN_VALU_HEAD=1 python bench.py $Q > "$OUT/valu.json"
timeout -k 10 300 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_diag_noload.so python bench.py $Q > "$OUT/noload.json"
timeout -k 10 300 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_diag_noload.so CCMI_SYN_VALU_HEAD=1 python bench.py $Q > "$OUT/noload_valu.json"
timeout -k 10 120 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_stamps.so python tools/prof_fused.py > "$OUT/stamps_mfma.txt"
timeout -k 10 120 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_stamps.so CCMI_SYN_VALU_HEAD=1 python tools/prof_fused.py > "$OUT/stamps_valu.txt"
echo done
