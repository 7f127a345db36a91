set -u
O=gpurun_out/r1d_ab; mkdir -p $O
Q="--steps 30 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
for i in 1 2 3; do
  timeout -k 10 120 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_base.so python bench.py $Q --serial > $O/base_serial_$i.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py $Q --serial > $O/new_serial_$i.json 2>/dev/null || exit 1
done
timeout -k 10 120 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_base.so python bench.py $Q > $O/base_overlap.json 2>/dev/null || exit 1
timeout -k 10 120 python bench.py $Q > $O/new_overlap.json 2>/dev/null || exit 1
timeout -k 10 120 env CCMI_LIB=$PWD/cool-chic_amd/lib/libccmi_stamps.so python tools/prof_fused.py > $O/stamps_new.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_forward.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_forward.log 2>&1 || exit 1
echo done
