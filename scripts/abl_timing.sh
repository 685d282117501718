#!/bin/bash
# In-kernel phase stamps of one Base step under the timing library and its two
# phase-ablation variants (common.h UNET_ABL: 1 = no MFMA, 2 = no pipelined DMA)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/image-segmentation-project_amd
for v in timing timing_abl1 timing_abl2; do
  echo "=== $v $(date +%T)"
  UNET_HIP_LIB=$L/libunet_hip_$v.so timeout -k 10 200 python3 scripts/conv_timing.py > gpurun_out/ct_$v.txt 2>&1 || { tail -5 gpurun_out/ct_$v.txt; exit 1; }
done
echo "=== done $(date +%T)"
