#!/bin/bash
# Step runner for GPU sessions (sourced on the GPU box, repo root), so a session is one
# gpurun command line instead of a one-off script:
#   gpurun -- 'source tools/gpu_lib.sh gpurun_out/r6a && run tests 600 $PT tests/test_decode_gpu.py && ab 3 lat ...'
# run NAME SECONDS CMD...   runs CMD from /tmp under its own time limit, output in $OUT/NAME.log;
#                           a failing step prints its tail and ends the session (no retries)
# ab N NAME SECONDS CMD...  N interleaved pairs: CMD against $ABLIB (tools/ablib/libccmi_base.so by default, as CCMI_LIB)
#                           and against the in-tree library -> NAME_base_i / NAME_new_i
# PT                        the GPU pytest command line (thread timeouts, stops at the first failure)
ROOT=$(pwd)
OUT=$ROOT/${1:-gpurun_out/session}
mkdir -p "$OUT"
export TMPDIR=/tmp
PT="python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --rootdir $ROOT"
run() {
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    (cd /tmp && timeout -k 10 "$secs" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    tail -2 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
ab() {
    local n=$1 name=$2 secs=$3
    shift 3
    for i in $(seq 1 "$n"); do
        run "${name}_base_$i" "$secs" env CCMI_LIB="${ABLIB:-$ROOT/tools/ablib/libccmi_base.so}" "$@"
        run "${name}_new_$i" "$secs" "$@"
    done
}
