#!/bin/bash
# full GPU suite, stem phase stamps, eager layer profile, convT dgrad tile sweep
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/image-segmentation-project_amd
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full2.log 2>&1; rc=$?
tail -1 gpurun_out/full2.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/full2.log | head -20; exit $rc; }
UNET_HIP_LIB=$L/libunet_hip_timing.so timeout -k 10 200 python3 scripts/conv_timing.py --filter input_conv 2>&1 | grep input_conv || exit 1
timeout -k 10 300 python3 scripts/tune_conv.py --only up1_dgrad,up2_dgrad --modes 0 --cfgs 0,3,5,10,11,12,14,21,22,24,1,4,6,8,16,17,19,23 --reps 3 2>&1 | grep -v amdgpu.ids || exit 1
