#!/bin/bash
# round 5: the level replay's chain snapshot kept and rebuilt every 4 batches (tests + A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5v_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5v "" "" incr_cfg2 new env:CRDTM_ILR_SNAP_EVERY=1 env:CRDTM_ILR_SNAP_EVERY=8 env:CRDTM_ILR_SNAP_EVERY=1000
