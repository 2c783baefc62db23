#!/bin/bash
# round 5: the whole GPU suite on the build with uniform regions left unstructured, then bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5m_tests.log; [ $rc = 0 ] || exit $rc
for w in cfg2 trees incr_cfg2 cfg1 deep10m_il; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample 0 --pmc off --verbose > gpurun_out/r5m_$w.log 2>&1 || { echo FAIL $w; tail -5 gpurun_out/r5m_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5m_$w.log | head -1)"
done
