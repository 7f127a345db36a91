#!/bin/bash
# Round 5 session zn: t_quant with 4 latents per thread --
# training + forward
# parity on the product library and on the side-stream spin build, step A/B against
# tools/ablib/r5zn_base.so, the isolated training trace.  Usage: bash tools/gpu_r5zn.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5zn}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run train_tests 900 $PT $ROOT/tests/test_train_gpu.py $ROOT/tests/test_mirror_train_gpu.py $ROOT/tests/test_api_mirror.py $ROOT/tests/test_rd_gpu.py -k "not full_schedule"
run fwd_tests 300 $PT $ROOT/tests/test_forward.py
for r in 1 2 3; do
  run step_base_$r 300 env CCMI_LIB=$ROOT/tools/ablib/r5zn_base.so python3 $ROOT/tools/bench_train.py 8 --no-cpu
  run step_new_$r 300 python3 $ROOT/tools/bench_train.py 8 --no-cpu
done
export CCMI_ARM_OVERLAP=0
run trace_iso 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_iso -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu
echo "all steps passed" | tee -a "$OUT/steps.log"
