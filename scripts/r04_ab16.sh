#!/bin/bash
# current build vs the library of commit c16c77e (ab/head_c16.so), interleaved; then the eager layer profile
set -o pipefail
bash scripts/ab_bench.sh 3 - UNET_HIP_LIB=$PWD/ab/head_c16.so || exit 1
timeout -k 10 200 python3 scripts/layer_profile.py --top 40 > gpurun_out/lp3.txt 2>&1 || exit 1
