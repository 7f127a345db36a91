#!/bin/bash
# Round 5 session a: side-stream join (pooled streams + SideJoin guard) -- training tests on the
# product library and on the diagnostic spin build (make -C cool-chic_amd spin), the decoder
# tests (pooled chunk streams), the smoke, and the decode stamps of the round-start chain.
# Usage (GPU box, repo root): bash tools/gpu_r5a.sh OUTDIR
set -u
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/r5a}
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
run train_tests_spin 600 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_spin.so $PT $ROOT/tests/test_train_gpu.py $ROOT/tests/test_mirror_train_gpu.py
run dec_tests 600 $PT $ROOT/tests/test_decode_gpu.py $ROOT/tests/test_codec_e2e.py
run smoke 300 python -c "import sys; sys.path.insert(0, '$ROOT'); import __graft_entry__ as g; g.smoke()"
for s in B-BQTerrace-lmbda-00001_1920x1080_50p_yuv420_8b.cool E-FourPeople-lmbda-00001_1280x720_60p_yuv420_8b.cool; do
  run stamps_${s%%_*} 300 env CCMI_LIB=$ROOT/cool-chic_amd/lib/libccmi_stamps.so python $ROOT/tools/prof_decode_one.py $s
done
run lat 300 python $ROOT/tools/decode_latency.py 2
echo "all steps passed" | tee -a "$OUT/steps.log"
