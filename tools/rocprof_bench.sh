#!/bin/bash
# Kernel trace + stats and HBM PMC passes of bench.py on the GPU box (run via gpurun).
# Writes under gpurun_out/prof_<tag>/ ; summarise with tools/summarise_prof.py.
set -euo pipefail
TAG=${1:-r1}
STEPS=${2:-10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --decode-reps 0 --hd-steps 0 --hd-decode-reps 0 > "$OUT/bench_trace.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --decode-reps 0 --hd-steps 0 --hd-decode-reps 0 > "$OUT/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$R/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --decode-reps 0 --hd-steps 0 --hd-decode-reps 0 > "$OUT/bench_write.json"
echo done
