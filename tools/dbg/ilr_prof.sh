#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
CRDTM_ILR_STATS=1 CRDTM_ILR_DEBUG=1 NB=3 timeout -k 10 300 python -u tools/dbg/ilr_prof.py > gpurun_out/ilr_prof.log 2>&1; rc=$?
grep -E "^ilr|^  L|^batch" gpurun_out/ilr_prof.log; exit $rc
