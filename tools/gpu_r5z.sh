#!/bin/bash
# round 5: gap heads found by the in-gap kernel (incremental flat): tests + A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5z_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5z "" "" incr new lib:abtest/prev/libcrdtm.so
