#!/bin/bash
# Bench line of every config (one box, graph replay) -> gpurun_out/configs.jsonl
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for args in "--attention" "--width 2" "--size 1024 --batch 4" "--backbone resnet50" "--width 2 --fp8" "--data --batch 256"; do
  echo "=== bench.py $args"
  timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  grep '^{' gpurun_out/cfg.log | tee -a gpurun_out/configs.jsonl | grep -o '"value": [0-9.]*'
done
