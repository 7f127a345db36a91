#!/bin/bash
# Training-step A/B: the training parity tests on the current library, then ms per
# iteration (tools/bench_train.py, 8 frames of 512x768) for the current library and
# tools/ablib/$1.  Usage (GPU box, repo root): bash tools/ab_train.sh OTHER OUTDIR
set -u
OTHER=$(pwd)/tools/ablib/$1
OUT=${2:-gpurun_out/abtrain}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py tests/test_quantize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 5 200 python tools/bench_train.py 8 > $OUT/new$r.log 2>&1 || exit 1
  timeout -k 5 200 env CCMI_LIB=$OTHER python tools/bench_train.py 8 > $OUT/other$r.log 2>&1 || exit 1
done
tail -n 2 $OUT/new*.log $OUT/other*.log
