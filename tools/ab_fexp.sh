set -u
OUT=gpurun_out/abfe; mkdir -p $OUT
timeout -k 10 300 python tools/rate_margin.py > $OUT/margin_cur.log 2>&1 && tail -1 $OUT/margin_cur.log && \
CCMI_LIB=$(pwd)/tools/ablib/libccmi_fexp.so timeout -k 10 300 python tools/rate_margin.py > $OUT/margin_fexp.log 2>&1 && tail -12 $OUT/margin_fexp.log && \
for v in cur fexp cur2 fexp2; do
  L=""; case $v in fexp*) L="CCMI_LIB=$(pwd)/tools/ablib/libccmi_fexp.so";; esac
  env $L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 0 > $OUT/$v.log 2>&1 || exit 1
  tail -c 3000 $OUT/$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['stage_ms_per_step'])"
done
