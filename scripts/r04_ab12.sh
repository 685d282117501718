#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
L=$PWD/image-segmentation-project_amd
for v in abl3 abl4; do echo "## $v"; UNET_HIP_LIB=$L/libunet_hip_timing_$v.so timeout -k 10 200 python3 scripts/conv_timing.py --filter enc1.0 2>&1 | grep -v amdgpu.ids || exit 1; done
echo "## abl3 wscfg4"; UNET_WSCFG=4 UNET_HIP_LIB=$L/libunet_hip_timing_abl3.so timeout -k 10 200 python3 scripts/conv_timing.py --filter enc1.0 2>&1 | grep -v amdgpu.ids || exit 1
UNET_WSCFG=4 timeout -k 10 200 python3 -u -m pytest tests/test_wiring_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "forward_ops or backward_ops" 2>&1 | tail -1
bash scripts/ab_bench.sh 2 - UNET_WSCFG=4 || exit 1
