#!/bin/bash
# Run GPU steps in order; stop at the first failing step (a test failure can
# be a GPU fault: start nothing more on the GPU after it).
# usage: scripts/gpu_check.sh "<name>:<timeout>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout $tmo) : $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
done
exit 0
