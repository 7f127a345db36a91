#!/bin/bash
# Window-size A/B of the fused decode kernel: builds libccmi variants whose
# syn_fused_kernel uses a taller window (fewer halo rows recomputed, fewer workgroups per CU)
# into tools/ablib/.  Build here:   bash tools/ab_fused_window.sh build
# Run on the GPU box:               bash tools/ab_fused_window.sh run OUTDIR
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS="rh48t768w6:48:768:6 rh64t1024w4:64:1024:4"
if [ "${1:-}" = build ]; then
    B=$ROOT/cool-chic_amd/build
    for v in $VARIANTS; do
        IFS=: read -r name rh th w <<< "$v"
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fwrapv --offload-arch=gfx950 -munsafe-fp-atomics \
            -DCCMI_FUSED_RH=$rh -DCCMI_FUSED_THREADS=$th -DCCMI_FUSED_WPE=$w -x hip \
            -c $ROOT/cool-chic_amd/csrc/fwd_syn.hip -o /tmp/fwd_syn_$name.o || exit 1
        objs=$(ls $B/*.o | grep -v '/fwd_syn.o$')
        /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/tools/ablib/$name.so $objs /tmp/fwd_syn_$name.o || exit 1
        echo built tools/ablib/$name.so
    done
    exit 0
fi
OUT=$ROOT/${2:-gpurun_out/abwin}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
QB="bench.py --steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-decode-reps 0 --hd-steps 20"
for v in $VARIANTS; do
    name=${v%%:*}
    timeout -k 10 300 env CCMI_LIB=$ROOT/tools/ablib/$name.so python -u -m pytest tests/test_forward.py -m gpu -x -q \
        --timeout 120 --timeout-method thread > $OUT/pytest_$name.log 2>&1 || { tail -30 $OUT/pytest_$name.log; exit 1; }
    echo "$name: $(tail -1 $OUT/pytest_$name.log)"
done
for r in 1 2; do
    timeout -k 10 200 python3 $QB > $OUT/base$r.log 2>&1 || exit 1
    for v in $VARIANTS; do
        name=${v%%:*}
        timeout -k 10 200 env CCMI_LIB=$ROOT/tools/ablib/$name.so python3 $QB > $OUT/${name}_$r.log 2>&1 || exit 1
    done
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    if "pytest" in f: continue
    l = [x for x in open(f) if x.startswith("{")]
    if not l: continue
    r = json.loads(l[-1])
    print(f.split("/")[-1], r["value"], r["stage_ms_per_step"], r["roofline"]["frac"],
          r["path_a_1080p"]["value"], r["path_a_1080p"]["stage_ms_per_step"])
PY
