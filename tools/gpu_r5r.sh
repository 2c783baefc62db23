#!/bin/bash
# round 5: grid caps of the flat kernels, second round (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_ab.sh r5r "" "" flat10m new env:CRDTM_MASK_GRID=768 env:CRDTM_MASK_GRID=1536 env:CRDTM_EX_GRID=4096 env:CRDTM_RUN_GRID=4096 env:CRDTM_NEXT_GRID=2048 env:CRDTM_NEXT_GRID=4096 env:CRDTM_PRE_GRID=384 env:CRDTM_CLAIM_GRID=1536
