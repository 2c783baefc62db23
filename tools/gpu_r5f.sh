#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_ab.sh r5f "" "" flat10m new env:CRDTM_FLAT_SPEC=0 "env:CRDTM_FLAT_SPEC=0 CRDTM_LIB=abtest/nt0/libcrdtm.so" lib:abtest/base/libcrdtm.so || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_prof_new -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --cpu-sample 0 --pmc off --profile-steps 0 > gpurun_out/r5f_prof_new.log 2>&1 || exit 1
CRDTM_LIB=abtest/base/libcrdtm.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_prof_base -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --cpu-sample 0 --pmc off --profile-steps 0 > gpurun_out/r5f_prof_base.log 2>&1
