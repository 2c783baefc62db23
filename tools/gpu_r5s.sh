#!/bin/bash
# round 5: 8-bit digit small radix sort (incremental flat), A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flat_closed_form or incremental_chain or failed_fresh" > gpurun_out/r5s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5s_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5s "" "" incr new env:CRDTM_RS_SMALL=1024
