#!/bin/bash
# round 5 final: the whole GPU suite, smoke, then the incremental flat bench line and trace (profiles)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5f_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f_smoke.log 2>&1 || { tail -5 gpurun_out/r5f_smoke.log; exit 1; }
tail -1 gpurun_out/r5f_smoke.log
for w in incr; do
  timeout -k 10 400 python3 -u bench.py --workload $w > gpurun_out/r5f_${w}_bench.log 2>&1 || exit 1
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f_${w}_bench.log | head -1)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off > gpurun_out/r5f_prof_$w.log 2>&1 || exit 1
done
