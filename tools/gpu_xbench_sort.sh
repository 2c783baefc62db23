#!/bin/bash
# The incremental gap sort's kernels on key distributions, among them one
# incr bench batch's gap keys (dumped on demand with the test hook
# CRDTM_FI_DUMP_KEYS, engine.h test_hooks()), then the incremental tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CRDTM_TEST_HOOKS=1 CRDTM_FI_DUMP_KEYS=gpurun_out/incr_keys.bin timeout -k 10 200 \
  python3 -u bench.py --workload incr --steps 1 --warmup 0 --cpu-sample 0 --pmc off > gpurun_out/xbench_dump.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/xbench_sort.py 10000 gpurun_out/incr_keys.bin > gpurun_out/xbench_sort.log 2>&1; rc=$?; cat gpurun_out/xbench_sort.log; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "closed_form or chain" > gpurun_out/xbench_sort_tests.log 2>&1
rc=$?; tail -3 gpurun_out/xbench_sort_tests.log; exit $rc
