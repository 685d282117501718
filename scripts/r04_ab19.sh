#!/bin/bash
set -o pipefail
bash scripts/ab_bench.sh 2 - UNET_APPLY_CAP_FWD=128 UNET_APPLY_CAP_FWD=192 || exit 1
