#!/bin/bash
# Round 5 session w: the training ARM's side stream at the least stream priority (CCMI_ARM_PRIO=1)
# with 1..3 ARM workgroups per CU (CCMI_ARM_OVERLAP) against the default (normal priority, 1 per
# CU); training parity on the low-priority form.  Usage: bash tools/gpu_r5w.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5w}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -1 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
PT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
run tests_prio 600 env CCMI_ARM_PRIO=1 $PT $ROOT/tests/test_train_gpu.py $ROOT/tests/test_mirror_train_gpu.py
B="$ROOT/tools/bench_train.py 8 --no-cpu"
for r in 1 2; do
  run s_def_$r 300 python3 $B
  run s_p1c1_$r 300 env CCMI_ARM_PRIO=1 CCMI_ARM_OVERLAP=1 python3 $B
  run s_p1c2_$r 300 env CCMI_ARM_PRIO=1 CCMI_ARM_OVERLAP=2 python3 $B
  run s_p1c3_$r 300 env CCMI_ARM_PRIO=1 CCMI_ARM_OVERLAP=3 python3 $B
  run s_p0c2_$r 300 env CCMI_ARM_OVERLAP=2 python3 $B
done
echo "all steps passed" | tee -a "$OUT/steps.log"
