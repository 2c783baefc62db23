#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CRDTM_ILR_DEBUG=1 timeout -k 10 120 python -u tools/dbg/c2shape_dbg.py > gpurun_out/r5b_dbg.log 2>&1
rc=$?; grep -v "^$" gpurun_out/r5b_dbg.log | tail -12; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_incremental.py tests/test_traversal.py tests/test_gpu_parity_gaps.py -m gpu -v --timeout 300 --timeout-method thread -k "incr_cfg2_bench_shape or sweep or commit_failure or refuse or guard_g_statistics_match" > gpurun_out/r5b_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5b_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --pmc off --verbose > gpurun_out/r5b_flat.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5b_flat.log; exit $rc
