#!/bin/bash
# GPU tests, then per-layer profile + bench of the in-tree library, and the
# bench of a baseline build (UNET_HIP_LIB) for comparison.  usage: scripts/ab_step.sh [base.so]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/tests.log | head -20; exit $rc; }
timeout -k 10 200 python3 scripts/layer_profile.py --all > gpurun_out/layer_now.txt 2>&1 || exit $?
head -16 gpurun_out/layer_now.txt
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_new.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/bench_new.log
if [ -n "$1" ]; then
  UNET_HIP_LIB=$1 timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/bench_base.log 2>&1 || exit $?
  echo -n "base "; grep -o '"value": [0-9.]*' gpurun_out/bench_base.log
fi
