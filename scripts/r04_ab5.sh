#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_bench.txt
bash scripts/abl_timing.sh || exit 1
for v in timing timing_abl1 timing_abl2; do echo "## $v"; grep "batch" gpurun_out/ct_$v.txt; done
bash scripts/ab_bench.sh 2 - UNET_WG_BATCH=0 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_wide_fp8_full_gpu.py tests/test_ddp_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k "wide_fp8 or share" > gpurun_out/newtests.log 2>&1; rc=$?
grep -E "passed|failed|Wide fp8|rank|Error|assert" gpurun_out/newtests.log | head -20
exit $rc
