#!/bin/bash
# Builds the t_sp_bwd<3> diagnostic variants (wrong results by design; timing only) into
# tools/ablib/spb_<variant>.so: NOLOAD (tile loads replaced by arithmetic), NODW (no weight-
# gradient MFMAs), NODX (no input-gradient arithmetic), NOBORDER (no border-tap fold; session
# r5zc traced it against the qrange border loops the fold replaced).
# Run on the CPU host; the GPU session traces each with bench_train.py.
set -e
cd "$(dirname "$0")/../cool-chic_amd"
SRC="csrc/*.hip csrc/*.cpp"
for v in NOLOAD NODW NODX NOBORDER; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fwrapv --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function \
    -DCCMI_DIAG_SPB_$v -shared -o ../tools/ablib/spb_$(echo $v | tr A-Z a-z).so -x hip $SRC &
done
wait
