#!/bin/bash
# eager per-launch breakdown + rocprofv3 stats of the graph-replayed bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/layer_profile.py --top 60 > gpurun_out/lp.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
tail -1 gpurun_out/prof_bench.log
