#!/bin/bash
# wgrad loader-wave kernel: GPU tests, phase stamps, A/B bench vs the old kernel
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_call.sh - UNET_WG_LD=0 - UNET_WG_LD=0 || exit $?
UNET_HIP_LIB=$PWD/image-segmentation-project_amd/libunet_hip_timing.so timeout -k 10 200 \
  python3 scripts/conv_timing.py > gpurun_out/ct_ld.txt 2>&1 || { tail -5 gpurun_out/ct_ld.txt; exit 1; }
echo done
