#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
L=$PWD/image-segmentation-project_amd
timeout -k 10 300 python3 -u -m pytest tests/test_wiring_gpu.py tests/test_bn_prologue_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/t11.log 2>&1; rc=$?
tail -2 gpurun_out/t11.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t11.log | head -20; exit $rc; }
UNET_HIP_LIB=$L/libunet_hip_timing_abl3.so timeout -k 10 200 python3 scripts/conv_timing.py --filter enc1.0 > gpurun_out/ct_abl3.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ct_abl3.txt
bash scripts/ab_bench.sh 2 - UNET_HIP_LIB=$PWD/ab/base_lib.so || exit 1
