#!/bin/bash
# One GPU round trip for this session's work: selected parity tests, then bench lines.
#   tools/gpu_round.sh <tag> "<pytest selection>" <workload> [<workload> ...]
set -o pipefail
T=$1; SEL=$2; shift 2
mkdir -p gpurun_out
if [ -n "$SEL" ]; then
  eval timeout -k 10 600 python -u -m pytest $SEL -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 \
    || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
  tail -3 gpurun_out/${T}_tests.log
fi
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample 0 --verbose > gpurun_out/${T}_$w.log 2>&1 \
    || { echo BENCH_FAIL $w; tail -20 gpurun_out/${T}_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_$w.log | head -1)"
done
