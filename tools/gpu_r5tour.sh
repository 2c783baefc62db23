#!/bin/bash
# round 5: gaps ordered by an Euler tour of their ops' tree (incr flat): incremental tests, A/B + trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5tour_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5tour_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5tour "" "" incr new lib:abtest/le/libcrdtm.so && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5tour_prof_incr -o run --output-format csv -- python3 bench.py --workload incr --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off > gpurun_out/r5tour_prof_incr.log 2>&1
