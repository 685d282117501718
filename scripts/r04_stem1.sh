#!/bin/bash
# stem backward rework: parity tests, then phase stamps and the eager layer profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/image-segmentation-project_amd
timeout -k 10 300 python -u -m pytest tests/test_stem_rc_gpu.py tests/test_wiring_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ts1.log 2>&1; rc=$?
tail -1 gpurun_out/ts1.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/ts1.log | head -20; exit $rc; }
UNET_HIP_LIB=$L/libunet_hip_timing.so timeout -k 10 200 python3 scripts/conv_timing.py --filter input_conv 2>&1 | grep input_conv || exit 1
timeout -k 10 200 python3 scripts/layer_profile.py --top 12 > gpurun_out/lp2.txt 2>&1 || exit 1
head -16 gpurun_out/lp2.txt
