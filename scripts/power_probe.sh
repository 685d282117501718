#!/bin/bash
# GPU power / clock while the bench runs (read-only amd-smi queries)
set -o pipefail
mkdir -p gpurun_out
( for i in $(seq 1 40); do amd-smi metric -p -c 2>/dev/null | grep -iE "SOCKET_POWER|GFX_0|POWER_LIMIT|CLK" | head -8; echo "--- $i"; sleep 0.5; done ) > gpurun_out/power.txt 2>&1 &
P=$!
timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 1500 --warmup 10 > gpurun_out/power_bench.log 2>&1
kill $P 2>/dev/null; wait $P 2>/dev/null
amd-smi static --limit 2>/dev/null | head -30 >> gpurun_out/power.txt
tail -1 gpurun_out/power_bench.log | grep -o '"value": [0-9.]*'
