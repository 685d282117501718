#!/bin/bash
# forward BN apply grid cap sweep (interleaved)
set -o pipefail
bash scripts/ab_bench.sh 2 - UNET_APPLY_CAP_FWD=512 UNET_APPLY_CAP_FWD=1024 UNET_APPLY_CAP_FWD=2048 || exit 1
