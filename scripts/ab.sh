#!/bin/bash
# Interleaved A/B of whole-step throughput (bench.py graph replay, no CPU
# baseline, no parity leg, STEPS timed steps, default 150): R rounds over the
# given variants, one bench process per variant per round, every other round in
# reverse order (ABBA), medians at the end.
# A variant is  [VAR=val[,VAR=val...]][@lib.so]  ("-" or "" = defaults, the
# in-tree libunet_hip.so); e.g.
#   scripts/ab.sh 3 - @ab/libunet_hip_r04.so UNET_APPLY_CAP=1024
#   BENCH_ARGS="--width 2" scripts/ab.sh 3 - UNET_NO_FL=1
# AB_LAYERS="<regex>": per-layer instead (scripts/layer_profile.py, HIP events
# around every launch), printing the matching launch lines of every variant
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$1; shift
out=gpurun_out/ab.txt
: > $out
STEPS=${STEPS:-150}
specs=("$@")
for r in $(seq 1 $R); do
  # ABBA: every other round in reverse order (clock / thermal drift cancels)
  order=("${specs[@]}")
  if [ $((r % 2)) -eq 0 ]; then order=(); for ((i=${#specs[@]}-1; i>=0; i--)); do order+=("${specs[$i]}"); done; fi
  for spec in "${order[@]}"; do
    envs=${spec%%@*}; lib=""
    [[ "$spec" == *@* ]] && lib=${spec#*@}
    [ "$envs" = "-" ] && envs=""
    args=()
    [ -n "$envs" ] && IFS=',' read -ra args <<< "$envs"
    [ -n "$lib" ] && args+=("UNET_HIP_LIB=$PWD/$lib")
    if [ -n "$AB_LAYERS" ]; then
      echo "=== round $r [$spec]" | tee -a $out
      env "${args[@]}" timeout -k 10 120 python3 scripts/layer_profile.py --top 400 > gpurun_out/ab_layers.log 2>&1 || exit 1
      grep -E "$AB_LAYERS" gpurun_out/ab_layers.log | tee -a $out
      continue
    fi
    v=$(env "${args[@]}" timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --steps $STEPS --warmup 20 \
        $BENCH_ARGS 2>/dev/null | grep -o '"value": [0-9.]*' | grep -o '[0-9.]*$') || exit 1
    echo "round $r [$spec] $v" | tee -a $out
  done
done
python3 - "$out" <<'PY'
import re, statistics, sys
vals = {}
for l in open(sys.argv[1]):
    m = re.match(r"round \d+ \[(.*)\] ([\d.]+)", l)
    if m: vals.setdefault(m.group(1), []).append(float(m.group(2)))
base = None
for k, v in vals.items():
    med = statistics.median(v)
    base = base or med
    print(f"{k:48s} median {med:8.1f}  min {min(v):8.1f}  max {max(v):8.1f}  n={len(v)}  {med / base:6.3f}x")
PY
