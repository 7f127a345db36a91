#!/bin/bash
# Round 4, session a: decode / dist GPU tests after the batch-decode host rework, the default
# bench line, and one 8-way shard (--as-rank) of the weak-scaled legs.
# Usage (GPU box, repo root): bash tools/gpu_r4a.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4a}
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
run pytest_dec 900 python -u -m pytest $ROOT/tests/test_dist.py $ROOT/tests/test_train_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread
run bench 600 python3 $ROOT/bench.py
run bench_as_rank3 600 python3 $ROOT/bench.py --as-rank 3 --as-world 8 --no-cpu-baseline --hd-steps 0 --no-single-stream
echo "all steps passed" | tee -a "$OUT/steps.log"
