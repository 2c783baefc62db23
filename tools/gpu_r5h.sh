#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5h_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5h "" "" flat10m new env:CRDTM_FLAT_SPEC=0 "env:CRDTM_FLAT_SPEC=0 CRDTM_MASK_DEVQ=1" env:CRDTM_FLAT_SORT=radix env:CRDTM_EP_COHERENT=1
