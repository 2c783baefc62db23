#!/bin/bash
# round 5: final profiles part 2 (forest, incremental) and the level replay's 16-byte event stores (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "level_replay or dict_incremental" > gpurun_out/r5w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5w_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5w "" "" incr_cfg2 new lib:abtest/prev/libcrdtm.so
