#!/bin/bash
# rocprofv3 kernel stats of the GPU training step (tools/bench_train.py) on the GPU box.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_train_${1:-r1}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/bench_train.py" ${2:-8} > "$OUT/bench.log" 2>&1
echo done
