#!/bin/bash
# stem by recompute, second cut: parity, phase stamps, layer profile, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
L=$PWD/image-segmentation-project_amd
timeout -k 10 300 python3 -u -m pytest tests/test_stem_rc_gpu.py tests/test_wiring_gpu.py -m gpu -x -q -s --timeout 200 \
  --timeout-method thread -k "stem or backward_ops" > gpurun_out/t_stem.log 2>&1; rc=$?
grep -E "passed|failed|fraction|largest|logits|Error|assert" gpurun_out/t_stem.log | head -30
[ $rc -eq 0 ] || exit $rc
UNET_HIP_LIB=$L/libunet_hip_timing.so timeout -k 10 200 python3 scripts/conv_timing.py --filter input_conv > gpurun_out/ct_stem.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ct_stem.txt
timeout -k 10 120 python3 scripts/layer_profile.py > gpurun_out/lp_stem.txt 2>&1 || exit 1
grep -E "input_conv|maxpool|launches" gpurun_out/lp_stem.txt | head -12
bash scripts/ab_bench.sh 2 - UNET_STEM_RC=0 || exit 1
