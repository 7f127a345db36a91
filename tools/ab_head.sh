set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_forward.py tests/test_api_mirror.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fh.log 2>&1
Q="--steps 20 --warmup 5 --no-cpu-baseline --decode-reps 0 --encode-images 0 --hd-steps 0 --hd-decode-reps 0"
timeout -k 10 300 python bench.py $Q > gpurun_out/ab_mfma1.json
timeout -k 10 300 env CCMI_SYN_VALU_HEAD=1 python bench.py $Q > gpurun_out/ab_valu1.json
timeout -k 10 300 python bench.py $Q > gpurun_out/ab_mfma2.json
timeout -k 10 300 env CCMI_SYN_VALU_HEAD=1 python bench.py $Q > gpurun_out/ab_valu2.json
