#!/bin/bash
# epilogue constants batched + stem by recompute: parity, phase stamps, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
L=$PWD/image-segmentation-project_amd
timeout -k 10 400 python3 -u -m pytest tests/test_stem_rc_gpu.py tests/test_wiring_gpu.py tests/test_kernels_gpu.py \
  tests/test_bn_prologue_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/t8.log 2>&1; rc=$?
tail -3 gpurun_out/t8.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t8.log | head -20; exit $rc; }
UNET_HIP_LIB=$L/libunet_hip_timing.so timeout -k 10 200 python3 scripts/conv_timing.py --filter input_conv > gpurun_out/ct_stem.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ct_stem.txt
UNET_HIP_LIB=$L/libunet_hip_timing_abl3.so timeout -k 10 200 python3 scripts/conv_timing.py --filter enc1.0 > gpurun_out/ct_abl3b.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ct_abl3b.txt
timeout -k 10 120 python3 scripts/layer_profile.py > gpurun_out/lp8.txt 2>&1 || exit 1
head -16 gpurun_out/lp8.txt; grep -E "input_conv|maxpool" gpurun_out/lp8.txt | head -8
bash scripts/ab_bench.sh 2 - UNET_HIP_LIB=$PWD/ab/base_lib.so UNET_STEM_RC=0 || exit 1
