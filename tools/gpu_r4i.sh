#!/bin/bash
# Round 4, sessions i / s: training-kernel ablations (tools/arm_diag.sh A16_* / LVL_* variants,
# wrong results by construction, timed only) -- kernel traces of tools/bench_train.py 8 per library.
# Usage: bash tools/gpu_r4i.sh OUTDIR LIB...
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4i}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
    name=$(basename $lib .so)
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 tools/bench_train.py 8 --no-cpu --lib $lib > "$OUT/$name.log" 2>&1
    rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
done
echo "all steps passed" | tee -a "$OUT/steps.log"
