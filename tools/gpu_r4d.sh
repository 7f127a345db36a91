#!/bin/bash
# Round 4, session d: the round-style session (tools/gpu_round.sh: every GPU test, the default
# bench line, kernel trace + HBM PMC passes), then the training-step A/B against round 3.
# Usage (GPU box, repo root): bash tools/gpu_r4d.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=${1:-gpurun_out/r4d}
TESTS="${TESTS:-}" bash tools/gpu_round.sh $OUT || exit $?
for r in 1 2; do
  timeout -k 10 200 python tools/bench_train.py 8 --no-cpu > $ROOT/$OUT/train_new$r.log 2>&1 || exit 1
  timeout -k 10 200 env CCMI_LIB=$ROOT/tools/ablib/r3base.so python tools/bench_train.py 8 --no-cpu > $ROOT/$OUT/train_r3_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python tools/bench_train.py 8 --no-cpu --default-arch > $ROOT/$OUT/train_def_new$r.log 2>&1 || exit 1
  timeout -k 10 200 env CCMI_LIB=$ROOT/tools/ablib/tarm2.so python tools/bench_train.py 8 --no-cpu --default-arch > $ROOT/$OUT/train_def_tarm2_$r.log 2>&1 || exit 1
done
tail -n1 $ROOT/$OUT/train_*.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/trace_train -o run -- python3 $ROOT/tools/bench_train.py 8 --no-cpu > $ROOT/$OUT/trace_train.log 2>&1 || exit 1
echo "r4d done"
