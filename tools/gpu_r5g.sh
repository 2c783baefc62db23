#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_gaps.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "speculation or flat or exact" > gpurun_out/r5g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5g_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5g "" "" flat10m new lib:abtest/ntn0/libcrdtm.so env:CRDTM_FLAT_SPEC=0 "env:CRDTM_FLAT_SPEC=0 CRDTM_LIB=abtest/ntn0/libcrdtm.so"
