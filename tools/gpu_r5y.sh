#!/bin/bash
# round 5: the incremental flat path with four launches fewer (gate in the window list, one superblock pass,
# the key index in the commit, the fold's counters cleared up front): tests + A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5y_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5y_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5y "" "" incr new lib:abtest/prev/libcrdtm.so
