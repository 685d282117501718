#!/bin/bash
# stem kernels with LDS-only barriers; ws epilogue store ablation (abl4)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
L=$PWD/image-segmentation-project_amd
timeout -k 10 300 python3 -u -m pytest tests/test_stem_rc_gpu.py tests/test_wiring_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "stem or backward_ops or forward_ops" > gpurun_out/t9.log 2>&1; rc=$?
tail -2 gpurun_out/t9.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t9.log | head -20; exit $rc; }
UNET_HIP_LIB=$L/libunet_hip_timing.so timeout -k 10 200 python3 scripts/conv_timing.py --filter input_conv > gpurun_out/ct_stem.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ct_stem.txt
for v in abl3 abl4; do
UNET_HIP_LIB=$L/libunet_hip_timing_$v.so timeout -k 10 200 python3 scripts/conv_timing.py --filter enc1.0 > gpurun_out/ct_$v.txt 2>&1 || exit 1
echo "## $v"; grep -v amdgpu.ids gpurun_out/ct_$v.txt
done
bash scripts/ab_bench.sh 2 - UNET_STEM_RC=0 || exit 1
