#!/bin/bash
# Round-4 baseline evidence in one box call: the default bench line, the
# in-kernel phase stamps of every conv launch (debug library), and the PMC
# wait/issue breakdown per kernel template (scripts/pmc_step.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== bench $(date +%T)"
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/b0_bench.log 2>&1 || { tail -5 gpurun_out/b0_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/b0_bench.log
echo "=== timing $(date +%T)"
UNET_HIP_LIB=$PWD/image-segmentation-project_amd/libunet_hip_timing.so timeout -k 10 200 \
  python3 scripts/conv_timing.py > gpurun_out/conv_timing.txt 2>&1 || { tail -5 gpurun_out/conv_timing.txt; exit 1; }
echo "=== pmc $(date +%T)"
bash scripts/pmc_step.sh || exit 1
echo "=== done $(date +%T)"
