#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5j_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5j "" "" flat10m new env:CRDTM_FL_NEXT=doc env:CRDTM_FLAT_SPEC=0 env:CRDTM_PRE_GRID=128 || exit 1
tools/gpu_ab.sh r5j "" "" incr new env:CRDTM_INCR_SORT=radix
