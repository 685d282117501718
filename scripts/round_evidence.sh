#!/bin/bash
# End-of-session GPU evidence in one box call (run from the repo root):
# GPU tests, smoke, the default bench line (with cpu_baseline), rocprofv3
# kernel stats + FETCH/WRITE + MFMA passes of the Base config, FETCH/WRITE of
# the HiRes config, the per-layer profile and every config's bench line.
# Stops at the first failing step.  Copy gpurun_out/ev_* and the summaries
# into profiles/<round>/<session>/ afterwards.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
step tests
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  > gpurun_out/ev_gpu_tests.txt 2>&1 || { tail -20 gpurun_out/ev_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/ev_gpu_tests.txt
step smoke
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/ev_gpu_tests.txt 2>&1 || exit 1
step profile_base
ROUND=${ROUND:-r03} bash scripts/profile_round.sh || exit 1
step pmc_hires
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_hr -o run \
  -- python3 scripts/layer_profile.py --top 3 --size 1024 --batch 4 > gpurun_out/pmc_fetch_hr.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_hr -o run \
  -- python3 scripts/layer_profile.py --top 3 --size 1024 --batch 4 > gpurun_out/pmc_write_hr.log 2>&1 || exit 1
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch_hr gpurun_out/pmc_write_hr gpurun_out/pmc_traffic_hires.json \
  --config "resnet34/w1/plain/bf16/4x1024" > gpurun_out/pmc_traffic_hires.txt || exit 1
# this build's traffic summaries where bench.py looks for them (box copy only;
# the same files are committed under profiles/ afterwards)
mkdir -p "profiles/${ROUND:-r03}/${SESSION:-s2}"
cp gpurun_out/pmc_traffic.json gpurun_out/pmc_traffic_hires.json "profiles/${ROUND:-r03}/${SESSION:-s2}/" || exit 1
step bench
timeout -k 10 300 python3 bench.py > gpurun_out/ev_bench.log 2>&1 || { tail -5 gpurun_out/ev_bench.log; exit 1; }
grep '^{' gpurun_out/ev_bench.log > gpurun_out/ev_bench.json
step layers
timeout -k 10 200 python3 scripts/layer_profile.py --all > gpurun_out/ev_layer_profile.txt 2>&1 || exit 1
step configs
bash scripts/bench_configs.sh || exit 1
step done
exit 0
