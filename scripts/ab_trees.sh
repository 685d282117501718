#!/bin/bash
# Interleaved A/B of whole-step throughput between this tree and another
# self-contained tree (its own bench.py, package and built library; e.g. an
# earlier round's commit built under ab/<name>/): R rounds, ABBA order,
# medians at the end.  Usage: scripts/ab_trees.sh R ab/r05
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$1; other=$2
out=gpurun_out/ab_trees.txt
: > $out
STEPS=${STEPS:-150}
run() {  # $1 = tree
  (cd "$1" && timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --steps $STEPS --warmup 20 2>/dev/null) \
    | grep -o '"value": [0-9.]*' | grep -o '[0-9.]*$'
}
for r in $(seq 1 $R); do
  order=(. "$other")
  [ $((r % 2)) -eq 0 ] && order=("$other" .)
  for t in "${order[@]}"; do
    v=$(run "$t") || exit 1
    echo "round $r [$t] $v" | tee -a $out
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
    print(f"{k:20s} median {med:8.1f}  min {min(v):8.1f}  max {max(v):8.1f}  n={len(v)}  {med / base:6.3f}x")
PY
