set -u
OUT=gpurun_out/abg; mkdir -p $OUT
Q="--steps 50 --warmup 10 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0"
timeout -k 10 300 python bench.py $Q > $OUT/graph.log 2>&1 && \
timeout -k 10 300 python bench.py $Q --no-graph > $OUT/eager.log 2>&1 && \
timeout -k 10 300 python bench.py $Q > $OUT/graph2.log 2>&1
rc=$?
for f in graph eager graph2; do tail -c 2500 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['eager'], d['stage_ms_per_step'])" ; done
exit $rc
