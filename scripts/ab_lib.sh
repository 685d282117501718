#!/bin/bash
# GPU tests (unless SKIP_TESTS=1), then the bench of the in-tree build
# alternating with a baseline build kept at ab/base_lib.so (git-ignored; copy
# the previous libunet_hip.so there first).  BENCH_ARGS: extra bench.py flags.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests.log 2>&1 || { tail -20 gpurun_out/tests.log; exit 1; }
  tail -1 gpurun_out/tests.log
fi
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/bn_$r.log 2>&1 || exit $?
  echo "new $(grep -o '"value": [0-9.]*' gpurun_out/bn_$r.log)"
  UNET_HIP_LIB=$PWD/ab/base_lib.so timeout -k 10 200 python3 bench.py --no-cpu-baseline $BENCH_ARGS \
    > gpurun_out/bb_$r.log 2>&1 || exit $?
  echo "base $(grep -o '"value": [0-9.]*' gpurun_out/bb_$r.log)"
done
