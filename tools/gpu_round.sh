#!/bin/bash
# Round-end style GPU session: full GPU test suite, default bench line, rocprofv3 kernel
# trace of the same bench command (profiles/), one PMC pass for HBM traffic.
# Usage (GPU box, repo root): bash tools/gpu_round.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
# TESTS: the test files to run, relative to the repo root (default: the whole suite)
if [ -n "${TESTS:-}" ]; then TESTS=$(for t in $TESTS; do printf '%s ' "$ROOT/$t"; done); else TESTS=$ROOT/tests; fi
run pytest_gpu 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread
run bench 600 python3 $ROOT/bench.py
QB="$ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python3 $QB
run pmc_size 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_size -- python3 $QB
run pmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -- python3 $QB
echo "all steps passed" | tee -a "$OUT/steps.log"
