#!/bin/bash
# Path B quick loop: decode parity, then single-stream latency new vs tools/ablib/libccmi_base.so.
# Usage (GPU box, repo root): bash tools/ab_dec_quick.sh OUTDIR
set -u
OUT=${1:-gpurun_out/dq}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 5 200 python tools/decode_latency.py 2 > $OUT/lat_new.log 2>&1 || exit 1
timeout -k 5 200 env CCMI_LIB=$PWD/tools/ablib/libccmi_base.so python tools/decode_latency.py 2 > $OUT/lat_base.log 2>&1 || exit 1
for v in new base; do python -c "import json; d=json.loads(open('$OUT/lat_$v.log').read().strip().splitlines()[-1]); print('$v', d['mean_ms'], d['max_ms'], d['all_md5_ok'], [r['ms'] for r in d['rows']])"; done
