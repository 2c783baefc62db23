#!/bin/bash
# round 5: the new parity tests, then a flat10m kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_incremental.py tests/test_traversal.py tests/test_gpu_parity_gaps.py -m gpu -x -v --timeout 300 --timeout-method thread -k "incr_cfg2_bench_shape or sweep or commit_failure or config2_shape or refuse or guard_g_statistics_match" > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5a_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --pmc off --verbose > gpurun_out/r5a_flat.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5a_flat.log; exit $rc
