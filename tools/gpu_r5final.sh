#!/bin/bash
# round 5: the whole GPU suite, smoke, then the incremental bench lines refreshed (profiles)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5f_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f_smoke.log 2>&1 || { tail -5 gpurun_out/r5f_smoke.log; exit 1; }
tail -1 gpurun_out/r5f_smoke.log
timeout -k 10 400 python3 -u bench.py --workload incr > gpurun_out/r5f_incr_bench.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f_incr_bench.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_prof_incr -o run --output-format csv -- python3 bench.py --workload incr --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off > gpurun_out/r5f_prof_incr.log 2>&1
