#!/bin/bash
# One GPU round trip: the full -m gpu suite, then 1-GPU bench lines (no CPU baseline).
#   tools/gpu_check.sh <tag> [workload ...]
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.log
[ $rc = 0 ] || exit $rc
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample 0 --pmc off --verbose > gpurun_out/${T}_$w.log 2>&1 \
    || { echo BENCH_FAIL $w; tail -20 gpurun_out/${T}_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_$w.log | head -1)"
done
