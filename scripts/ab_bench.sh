#!/bin/bash
# Interleaved A/B of whole-step throughput: R rounds x the given env settings,
# one bench process each (graph replay, no CPU baseline); prints every value
# and the per-setting median.   usage: scripts/ab_bench.sh R "VAR=V[,VAR2=V2]" ...   ("-" = defaults)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$1; shift
envs() { [ "$1" = "-" ] && return; echo "$1" | tr ',' ' '; }
for r in $(seq 1 $R); do
  i=0
  for kv in "$@"; do
    i=$((i+1))
    v=$(env $(envs "$kv") timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --steps 30 --warmup 10 2>/dev/null \
        | grep -o '"value": [0-9.]*' | grep -o '[0-9.]*$') || exit 1
    echo "round $r setting $i [$kv] $v" | tee -a gpurun_out/ab_bench.txt
  done
done
python3 - "$@" <<'PY'
import re, statistics, sys
vals = {}
for l in open("gpurun_out/ab_bench.txt"):
    m = re.match(r"round \d+ setting (\d+) \[(.*)\] ([\d.]+)", l)
    if m: vals.setdefault(m.group(2), []).append(float(m.group(3)))
for k, v in vals.items(): print(f"{k:40s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  max {max(v):8.1f}  n={len(v)}")
PY
