#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_gaps.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5i_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5i_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5i "" "" flat10m new env:CRDTM_EP_COHERENT=1 env:CRDTM_FLAT_SPEC=0 "env:CRDTM_FLAT_SPEC=0 CRDTM_MASK_DEVQ=1" env:CRDTM_PRE_BLIND=1 env:CRDTM_PRE_GRID=256
