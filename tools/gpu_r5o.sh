#!/bin/bash
# round 5: incremental flat commit gated on the device (one host round trip per batch), level-replay fills
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_parity.py tests/test_gpu_parity_gaps.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5o_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5o "" "" incr new lib:abtest/prev/libcrdtm.so || exit 1
tools/gpu_ab.sh r5o "" "" incr_cfg2 new lib:abtest/prev/libcrdtm.so
