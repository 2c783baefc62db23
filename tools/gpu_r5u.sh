#!/bin/bash
# round 5: forest replay sub-variants; deep10m level kernel occupancy / grid (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_ab.sh r5u "" "" trees new lib:abtest/fe/libcrdtm.so lib:abtest/fh/libcrdtm.so || exit 1
tools/gpu_ab.sh r5u "" "" deep10m new env:CRDTM_LV_LDS=20000 env:CRDTM_LV_LDS=60000 env:CRDTM_LV_LDS=8 env:CRDTM_LV_GRID=2048 env:CRDTM_LV_GRID=8192
