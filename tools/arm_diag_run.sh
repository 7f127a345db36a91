#!/bin/bash
# GPU box: kernel trace of tools/bench_train.py (B frames) for libccmi and each diagnostic
# variant built by tools/arm_diag.sh.  Usage: bash tools/arm_diag_run.sh OUTDIR [B]
set -eu
R=$(pwd)
OUT=$R/${1:-gpurun_out/armdiag}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${ARM_DIAG_VARIANTS:-base NOBIAS NOOUTER NOSCATTER NOLDSATOM NOGATOM}; do
    lib=$R/cool-chic_amd/lib/libccmi.so
    extra=""
    case $v in
        base) ;;
        VALU) extra="CCMI_ARM_VALU=1" ;;  # the VALU training ARM of the same library
        *) lib=$R/cool-chic_amd/lib/libccmi_arm_$v.so ;;
    esac
    (cd /tmp && { [ -z "$extra" ] || export $extra; } && CCMI_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run \
        -- python3 "$R/tools/bench_train.py" ${2:-8}) > "$OUT/$v.log" 2>&1
done
echo done
