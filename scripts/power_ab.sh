#!/bin/bash
# average socket power (read-only amd-smi samples) during a long bench run per setting
set -o pipefail
mkdir -p gpurun_out
envs() { [ "$1" = "-" ] && return; echo "$1" | tr ',' ' '; }
for kv in "$@"; do
  ( for i in $(seq 1 30); do amd-smi metric -p 2>/dev/null | grep -o "SOCKET_POWER: [0-9]*" ; sleep 0.3; done ) > gpurun_out/pw.txt 2>&1 &
  P=$!
  v=$(env $(envs "$kv") timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 2500 --warmup 20 2>/dev/null | grep -o '"value": [0-9.]*')
  kill $P 2>/dev/null; wait $P 2>/dev/null
  echo "[$kv] $v power: $(grep -o '[0-9]*$' gpurun_out/pw.txt | sort -n | tail -12 | tr '\n' ' ')"
done
