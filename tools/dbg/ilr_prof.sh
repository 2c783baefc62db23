#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ilr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ilr_tests.log; [ $rc = 0 ] || exit $rc
CRDTM_ILR_STATS=1 CRDTM_ILR_DEBUG=1 NB=3 timeout -k 10 300 python -u tools/dbg/ilr_prof.py > gpurun_out/ilr_prof.log 2>&1; rc=$?
grep -E "^ilr|^  L|^batch|k_ilr_prep|k_ilr_level" gpurun_out/ilr_prof.log; exit $rc
