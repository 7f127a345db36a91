#!/bin/bash
# Diagnostic variants of the training ARM kernel (container side): each drops one part of
# t_arm (bias MFMAs / weight-gradient MFMAs / context-gradient scatter), giving an upper
# bound on what that part costs.  Results are wrong by construction; never benchmarked as
# results.  Usage (cool-chic_amd/): bash ../tools/arm_diag.sh   -> lib/libccmi_arm_<v>.so
set -eu
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fwrapv --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-function"
OTHERS=$(ls build/*.o | grep -v '/train.o$')
for v in ${ARM_DIAG_VARIANTS:-NOBIAS NOOUTER NOSCATTER NOLDSATOM NOGATOM}; do  # t_arm16: A16_NORATE A16_NOOUTER A16_NOGATHER; t_lvl_bwd: LVL_NOREF LVL_NOUP LVL_NODW
    $CXX -DCCMI_DIAG_$( [[ $v == A16_* || $v == LVL_* ]] && echo "" || echo ARM_)$v -x hip -c csrc/train.hip -o build/diag_train_$v.obj
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libccmi_arm_$v.so $OTHERS build/diag_train_$v.obj
done
