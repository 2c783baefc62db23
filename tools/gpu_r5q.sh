#!/bin/bash
# round 5: NSR top level (incremental flat), grid caps of the flat kernels (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flat_closed_form or incremental_chain or failed_fresh" > gpurun_out/r5q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5q_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5q "" "" incr new lib:abtest/prev/libcrdtm.so || exit 1
tools/gpu_ab.sh r5q "" "" flat10m env:CRDTM_MASK_GRID=1024 env:CRDTM_MASK_GRID=512 "env:CRDTM_MASK_GRID=1024 CRDTM_MASK_U=1" "env:CRDTM_MASK_GRID=1024 CRDTM_RUN_GRID=1024" "env:CRDTM_MASK_GRID=1024 CRDTM_EX_GRID=1024" "env:CRDTM_MASK_GRID=1024 CRDTM_CLAIM_GRID=1024" "env:CRDTM_MASK_GRID=1024 CRDTM_HEADS_GRID=1024"
