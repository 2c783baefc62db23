#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 200 --timeout-method thread -k "adversarial" > gpurun_out/r5d_adv.log 2>&1
rc=$?; tail -3 gpurun_out/r5d_adv.log; [ $rc = 0 ] || exit $rc
exec_ab() { tools/gpu_ab.sh "$@"; }
tools/gpu_ab.sh r5d "tests/" "" flat10m new lib:abtest/nt0/libcrdtm.so lib:abtest/base/libcrdtm.so env:CRDTM_FLAT_SPEC=0
