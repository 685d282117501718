#!/bin/bash
# A/B a tuning environment variable over the per-layer profile with extra args:
# usage: scripts/ab_env2.sh VAR "v1 v2 ..." "<grep pattern>" [layer_profile args...]
var=$1; vals=$2; pat=$3; shift 3
for v in $vals; do
  echo "=== $var=$v"
  if [ "$v" = "unset" ]; then pre="env -u $var"; else pre="env $var=$v"; fi
  $pre timeout -k 10 120 python scripts/layer_profile.py --top 400 "$@" > gpurun_out/ab_$v.log 2>&1 || { echo "rc=$? at $v"; exit 1; }
  grep -E "$pat" gpurun_out/ab_$v.log
done
