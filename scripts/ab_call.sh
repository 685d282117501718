#!/bin/bash
# One A/B GPU call: GPU tests under the first setting, then the per-layer
# profile and bench of every setting.
# usage: scripts/ab_call.sh "VAR=V[,VAR2=V2]" "VAR=V" ...   ("-" = defaults)
set -o pipefail
mkdir -p gpurun_out
envs() { [ "$1" = "-" ] && return; echo "$1" | tr ',' ' '; }
first=$1
env $(envs "$first") timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/ab_tests.log | head -20; exit $rc; }
i=0
for kv in "$@"; do
  i=$((i+1))
  echo "=== [$i] $kv"
  env $(envs "$kv") timeout -k 10 200 python3 scripts/layer_profile.py --all > gpurun_out/ab_layers_$i.txt 2>&1 || exit $?
  head -8 gpurun_out/ab_layers_$i.txt
  env $(envs "$kv") timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_bench_$i.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/ab_bench_$i.log
done
exit 0
