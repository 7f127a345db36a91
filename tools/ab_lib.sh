#!/bin/bash
# A/B of libccmi builds: path-A parity tests on the current library, then the quick bench
# (path A only) alternating the current library and tools/ablib/$1.
# Usage (GPU box, repo root): bash tools/ab_lib.sh OTHER_LIB_NAME OUTDIR
set -u
OTHER=$(pwd)/tools/ablib/$1
OUT=${2:-gpurun_out/ablib}
mkdir -p "$OUT"
step() { # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
Q="--steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 10"
step pytest_fwd 400 python -u -m pytest tests/test_forward.py tests/test_api_mirror.py tests/test_codec_e2e.py -m gpu -x -q --timeout 200 --timeout-method thread
step bench_new 300 python bench.py $Q
step bench_other 300 env CCMI_LIB=$OTHER python bench.py $Q
step bench_new2 300 python bench.py $Q
step bench_other2 300 env CCMI_LIB=$OTHER python bench.py $Q
for f in bench_new bench_other bench_new2 bench_other2; do
  tail -c 3000 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$f', d['value'], d['stage_ms_per_step'], d['roofline']['frac'], d['path_a_1080p']['stage_ms_per_step'])" | tee -a "$OUT/steps.log"
done
