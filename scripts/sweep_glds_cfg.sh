#!/bin/bash
# Per-layer timing of every implicit-GEMM tile configuration (UNET_CONV_CFG
# override, applied to all glds-routed layers of the step) -> gpurun_out/cfg_<k>.txt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/layer_profile.py --all "$@" > gpurun_out/cfg_0.txt 2>&1 || exit $?
for k in $(seq 1 25); do
  UNET_CONV_CFG=$k timeout -k 10 120 python3 scripts/layer_profile.py --all "$@" > gpurun_out/cfg_$k.txt 2>&1 || exit $?
  echo "cfg $k done"
done
