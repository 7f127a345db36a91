#!/bin/bash
# Round 5 session zm: the whole GPU test suite and the smoke on the final code.  Usage: bash tools/gpu_r5zm.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5zm}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 900 python -u -m pytest $ROOT/tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
cd $ROOT && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
