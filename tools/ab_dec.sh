#!/bin/bash
# Path B check: bit-exact decode tests, then the bench's bit-exact decode legs only.
# Usage (GPU box, repo root): bash tools/ab_dec.sh OUTDIR
set -u
OUT=${1:-gpurun_out/abd}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_encode.py tests/test_codec_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --encode-images 0 --hd-steps 0 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -c 4000 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); [print(k, {x: d[k][x] for x in ('value_kernels','stage_ms','bit_exact_vs_reference_md5')}) for k in ('bitexact_decode','bitexact_decode_1080p')]"
