#!/bin/bash
# Path B: per-segment s_memtime stamps (diagnostic builds tools/ablib/st_new.so, st_base.so) on
# two class-E streams, then the single-stream latency of the current library and of
# tools/ablib/libccmi_base.so.  Usage (GPU box, repo root): bash tools/ab_dec_st.sh OUTDIR
set -u
OUT=${1:-gpurun_out/st}
mkdir -p "$OUT"
for v in new base; do
  for lm in 00001 0004; do
    CCMI_LIB=$PWD/tools/ablib/st_$v.so timeout -k 5 100 python tools/prof_decode_one.py E-FourPeople-lmbda-${lm}_1280x720_60p_yuv420_8b.cool > $OUT/${v}_$lm.log 2>&1 || exit 1
  done
done
grep "STAMPS stream 0\|arm_cabac" $OUT/*.log
timeout -k 5 200 python tools/decode_latency.py 2 > $OUT/lat_new.log 2>&1 || exit 1
timeout -k 5 200 env CCMI_LIB=$PWD/tools/ablib/libccmi_base.so python tools/decode_latency.py 2 > $OUT/lat_base.log 2>&1 || exit 1
for v in new base; do python -c "import json; d=json.loads(open('$OUT/lat_$v.log').read().strip().splitlines()[-1]); print('$v', d['mean_ms'], d['max_ms'], d['all_md5_ok'], [r['ms'] for r in d['rows']])"; done
