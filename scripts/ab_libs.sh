#!/bin/bash
# Interleaved A/B of whole-step throughput between library builds: R rounds x
# the given .so files ("-" = the in-tree libunet_hip.so), one bench process each
# (graph replay, no CPU baseline, no parity leg).
# usage: scripts/ab_libs.sh R lib1.so lib2.so ...   [BENCH_ARGS="--width 2"]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$1; shift
: > gpurun_out/ab_libs.txt
for r in $(seq 1 $R); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset UNET_HIP_LIB; else export UNET_HIP_LIB=$PWD/$lib; fi
    v=$(timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --steps 30 --warmup 10 $BENCH_ARGS 2>/dev/null \
        | grep -o '"value": [0-9.]*' | grep -o '[0-9.]*$') || exit 1
    echo "round $r [$lib] $v" | tee -a gpurun_out/ab_libs.txt
  done
done
unset UNET_HIP_LIB
python3 - <<'PY'
import re, statistics
vals = {}
for l in open("gpurun_out/ab_libs.txt"):
    m = re.match(r"round \d+ \[(.*)\] ([\d.]+)", l)
    if m: vals.setdefault(m.group(1), []).append(float(m.group(2)))
for k, v in vals.items(): print(f"{k:40s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  max {max(v):8.1f}  n={len(v)}")
PY
