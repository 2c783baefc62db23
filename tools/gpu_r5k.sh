#!/bin/bash
# round 5: structured forest replay (k_forest_wave_s), the path range check
# folded into the level kernels, the 1024-thread small radix sort -- parity,
# then A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_gaps.py tests/test_gpu_fullsize_parity.py tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "forest or trees or out_of_range or deep or incremental_chain or flat_closed_form or failed_fresh" > gpurun_out/r5k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5k_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5k "" "" trees new env:CRDTM_FOREST_WAVE=v lib:abtest/su/libcrdtm.so "env:CRDTM_FOREST_WAVE=v CRDTM_LIB=abtest/su/libcrdtm.so" || exit 1
tools/gpu_ab.sh r5k "" "" incr new env:CRDTM_RS_SMALL=512 || exit 1
tools/gpu_ab.sh r5k "" "" deep10m new lib:abtest/head/libcrdtm.so
