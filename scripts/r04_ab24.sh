#!/bin/bash
# tap-per-block batch reduce: full GPU suite, A/B vs ab/prev.so, rocprofv3 stats of the reduce
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full4.log 2>&1; rc=$?
tail -1 gpurun_out/full4.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/full4.log | head -20; exit $rc; }
bash scripts/ab_bench.sh 2 - UNET_HIP_LIB=$PWD/ab/prev.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof24 -o b \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/prof24.log 2>&1 || exit 1
