#!/bin/bash
# round 5: NSR queries four per wave (k_fi_gap4); run-mask unroll / grid A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flat_closed_form or incremental_chain or failed_fresh" > gpurun_out/r5p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5p_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5p "" "" incr new env:CRDTM_FI_GAP=64 || exit 1
tools/gpu_ab.sh r5p "" "" flat10m new env:CRDTM_MASK_U=1 env:CRDTM_MASK_U=4 env:CRDTM_MASK_GRID=4096 env:CRDTM_MASK_GRID=1024
