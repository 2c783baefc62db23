#!/bin/bash
# round 5: k_fi_gaps grid sweep (incr flat)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_ab.sh r5gg "" "" incr new env:CRDTM_GAPS_GRID=512 env:CRDTM_GAPS_GRID=1024 env:CRDTM_GAPS_GRID=4096 env:CRDTM_GAPS_GRID=10000
