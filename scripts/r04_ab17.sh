#!/bin/bash
# head backward with two pixels in flight: model tests, A/B vs ab/prev.so, layer profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_wiring_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t17.log 2>&1; rc=$?
tail -1 gpurun_out/t17.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t17.log | head -20; exit $rc; }
bash scripts/ab_bench.sh 2 - UNET_HIP_LIB=$PWD/ab/prev.so || exit 1
timeout -k 10 200 python3 scripts/layer_profile.py --top 12 > gpurun_out/lp4.txt 2>&1 || exit 1
grep head_bwd gpurun_out/lp4.txt
