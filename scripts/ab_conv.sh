#!/bin/bash
# A/B timing of the conv kernels: the in-tree library vs experimental builds
# (UNET_HIP_LIB), same shapes.  usage: SHAPES=a,b MODES=0,1 scripts/ab_conv.sh <exp.so> ...
set -o pipefail
mkdir -p gpurun_out
SH=${SHAPES:-enc3_3x3}; MO=${MODES:-0,1}
echo BASE; timeout -k 10 120 python3 scripts/tune_conv.py --reps 7 --cfgs 0 --only $SH --modes $MO --epi 2>&1 | grep -v amdgpu.ids || exit $?
for L in "$@"; do
  echo "EXP $L"; UNET_HIP_LIB=$L timeout -k 10 120 python3 scripts/tune_conv.py --reps 7 --cfgs 0 --only $SH --modes $MO --epi 2>&1 | grep -v "amdgpu.ids\|differ" || exit $?
done
