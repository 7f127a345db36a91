#!/bin/bash
# Training-kernel A/B (GPU box): parity tests, then kernel traces of tools/bench_train.py under
# each environment line of the list below.  Usage: bash tools/ab_train_nb.sh OUT
set -u
R=$(pwd); OUT=$R/${1:-gpurun_out/ab_train}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_mirror_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
i=0
while read -r E; do
  i=$((i+1))
  timeout -k 10 200 env $E rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$i -o run -- python3 $R/tools/bench_train.py 8 > $OUT/v$i.log 2>&1 || exit 1
  python3 - $OUT/v$i/run_kernel_stats.csv "$E" <<'PY'
import csv,sys,re
out={}
for r in csv.DictReader(open(sys.argv[1])):
    m=re.search(r'(t_\w+)(<[^>]*>)?', r['Name'])
    if m and m.group(1) in ('t_sp_bwd','t_arm16','t_head_bwd','t_head_fwd'): out[m.group(0)]=round(float(r['AverageNs'])/1e3,1)
print(sys.argv[2], out)
PY
done < ${VARIANTS:-$R/tools/ab_train_nb.txt}
