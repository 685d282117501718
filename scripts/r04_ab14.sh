#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
L=$PWD/image-segmentation-project_amd
timeout -k 10 300 python3 -u -m pytest tests/test_stem_rc_gpu.py tests/test_wiring_gpu.py tests/test_bn_prologue_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/t14.log 2>&1; rc=$?
tail -1 gpurun_out/t14.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t14.log | head -20; exit $rc; }
UNET_HIP_LIB=$L/libunet_hip_timing.so timeout -k 10 200 python3 scripts/conv_timing.py --filter "fwd" 2>&1 | grep -E "enc1.0|decoder1|decoder2.3" || exit 1
bash scripts/ab_bench.sh 2 - UNET_WS_SPLIT=0 || exit 1
