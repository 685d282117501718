#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/ab_tests.log | head -30; exit $rc; }
bash scripts/ab_bench.sh 3 - UNET_WG_BATCH=0 || exit 1
timeout -k 10 200 python3 scripts/layer_profile.py --all > gpurun_out/lp_batch.txt 2>&1 || exit 1
head -16 gpurun_out/lp_batch.txt
UNET_HIP_LIB=$PWD/image-segmentation-project_amd/libunet_hip_timing.so timeout -k 10 200 \
  python3 scripts/conv_timing.py > gpurun_out/ct_batch.txt 2>&1 || { tail -5 gpurun_out/ct_batch.txt; exit 1; }
grep batch gpurun_out/ct_batch.txt
