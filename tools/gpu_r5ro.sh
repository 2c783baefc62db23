#!/bin/bash
# round 5: the replica output in the last k_rep_max workgroup: the whole GPU suite, A/B on incr and incr_cfg2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ro_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5ro_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5ro "" "" incr new lib:abtest/jf/libcrdtm.so
