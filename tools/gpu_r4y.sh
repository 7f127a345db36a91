#!/bin/bash
# Round 4, session y: t_head_bwd record area sized to its instantiation (32,000 B per workgroup
# instead of 32,768), so five workgroups per CU fit: training parity tests, then kernel traces of
# the new build (occupancy-query grid), the same code capped at 4 per CU (tools/ablib/hbcap4.so)
# and the committed library (tools/ablib/r4u.so).  Usage: bash tools/gpu_r4y.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r4y}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
run pytest_train 600 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  run new$r 200 python tools/bench_train.py 8 --no-cpu
  run cap4_$r 200 python tools/bench_train.py 8 --no-cpu --lib $ROOT/tools/ablib/hbcap4.so
  run r4u_$r 200 python tools/bench_train.py 8 --no-cpu --lib $ROOT/tools/ablib/r4u.so
done
run trace_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- python3 tools/bench_train.py 8 --no-cpu
run trace_train_cap4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_cap4 -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/hbcap4.so
run trace_train_r4u 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_r4u -o run -- python3 tools/bench_train.py 8 --no-cpu --lib tools/ablib/r4u.so
echo "all steps passed" | tee -a "$OUT/steps.log"
