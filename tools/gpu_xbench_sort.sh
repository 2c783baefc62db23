#!/bin/bash
# The incremental gap sort's kernels on key distributions (tools/incr_keys.bin: one incr bench batch's keys,
# dumped with CRDTM_FI_DUMP_KEYS), then the incremental tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/xbench_sort.py 10000 tools/incr_keys.bin > gpurun_out/xbench_sort.log 2>&1; rc=$?; cat gpurun_out/xbench_sort.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "closed_form or chain" > gpurun_out/xbench_sort_tests.log 2>&1
rc=$?; tail -3 gpurun_out/xbench_sort_tests.log; exit $rc
