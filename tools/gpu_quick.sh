#!/bin/bash
# Focused GPU round trip: named test files first (fail fast), then bench lines.
#   tools/gpu_quick.sh <tag> "<test files>" [workload ...]
set -o pipefail
T=$1; F=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.log
[ $rc = 0 ] || exit $rc
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample 0 --pmc off --verbose > gpurun_out/${T}_$w.log 2>&1 \
    || { echo BENCH_FAIL $w; tail -20 gpurun_out/${T}_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_$w.log | head -1)"
done
