#!/bin/bash
# stem backward rework vs the committed library (ab/head_c16.so), interleaved
set -o pipefail
bash scripts/ab_bench.sh 3 - UNET_HIP_LIB=$PWD/ab/head_c16.so || exit 1
