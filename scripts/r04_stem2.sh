#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash scripts/r04_stem1.sh || exit 1
timeout -k 10 300 python3 scripts/tune_conv.py --only up1_dgrad,up2_dgrad --modes 0 --cfgs 0,3,5,10,11,12,14,21,22,24,1,4,6,8,16,17,19,23 --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
