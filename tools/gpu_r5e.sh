#!/bin/bash
# Round 5 session e: training tests, the isolated training-kernel trace (CCMI_ARM_OVERLAP=0:
# every kernel alone; the bench line's per-kernel training rooflines read it), then the
# default bench line.  Usage (GPU box, repo root): bash tools/gpu_r5e.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5e}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run train_tests 600 $PT $ROOT/tests/test_train_gpu.py $ROOT/tests/test_mirror_train_gpu.py
export CCMI_ARM_OVERLAP=0
run step_iso 300 python $ROOT/tools/bench_train.py 8 --no-cpu
run trace_iso 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_iso -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
unset CCMI_ARM_OVERLAP
run step 300 python $ROOT/tools/bench_train.py 8 --no-cpu
run bench 900 python3 $ROOT/bench.py
echo "all steps passed" | tee -a "$OUT/steps.log"
