#!/bin/bash
# stem by recompute: parity tests, A/B against the stored-y0 stem, layer profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
timeout -k 10 400 python3 -u -m pytest tests/test_stem_rc_gpu.py tests/test_wiring_gpu.py tests/test_ddp_gpu.py tests/test_dataset_gpu.py \
  tests/test_model_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread \
  -k "stem or backward_ops or forward_ops or share or reproducible or resize or upscale" > gpurun_out/t_stem.log 2>&1; rc=$?
grep -E "passed|failed|rel|fraction|largest|x1|d.x1|bn1|input_conv|rank [01]:|Error|assert" gpurun_out/t_stem.log | head -60
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh 3 - UNET_STEM_RC=0 || exit 1
timeout -k 10 120 python3 scripts/layer_profile.py > gpurun_out/lp_stem.txt 2>&1 || exit 1
grep -E "stem|input_conv|maxpool|launches" gpurun_out/lp_stem.txt | head -20
L=$PWD/image-segmentation-project_amd
UNET_HIP_LIB=$L/libunet_hip_timing_abl3.so timeout -k 10 200 python3 scripts/conv_timing.py --filter enc1 > gpurun_out/ct_abl3.txt 2>&1 || exit 1
UNET_HIP_LIB=$L/libunet_hip_timing_abl3.so timeout -k 10 200 python3 scripts/conv_timing.py --filter decoder1 >> gpurun_out/ct_abl3.txt 2>&1 || exit 1
cat gpurun_out/ct_abl3.txt | grep -v amdgpu.ids
