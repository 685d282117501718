#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   1. --kernel-trace --stats of a short bench run      -> gpurun_out/prof_bench
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (eager step) -> gpurun_out/pmc_fetch|pmc_write
#   4. MFMA pass (SQ_VALU_MFMA_BUSY_CYCLES, MOPS_BF16, GRBM_GUI_ACTIVE) -> gpurun_out/pmc_mfma
# then scripts/pmc_traffic.py turns 2+3 into gpurun_out/pmc_traffic.json and
# scripts/pmc_mfma.py turns 4 into gpurun_out/pmc_mfma.json.  Only
# gpurun_out/ comes back from the box: copy the summaries into profiles/ after.
set -o pipefail
export TMPDIR=/tmp
R=${ROUND:-r02}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run \
  -- python3 scripts/layer_profile.py --top 3 $LP_ARGS > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run \
  -- python3 scripts/layer_profile.py --top 3 $LP_ARGS > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json --config "${PMC_CONFIG:-resnet34/w1/plain/bf16/16x512}" \
  > gpurun_out/pmc_traffic.txt
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_mfma -o run \
  -- python3 scripts/layer_profile.py --top 3 > gpurun_out/pmc_mfma.log 2>&1 || exit $?
python3 scripts/pmc_mfma.py gpurun_out/pmc_mfma gpurun_out/pmc_mfma.json > gpurun_out/pmc_mfma.txt
