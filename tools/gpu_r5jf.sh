#!/bin/bash
# round 5: the jump hops fused into the gap search (incr flat): incremental tests, A/B + trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread -k "closed_form or chain" > gpurun_out/r5jf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5jf_tests.log; [ $rc = 0 ] || exit $rc
tools/gpu_ab.sh r5jf "" "" incr new lib:abtest/rv/libcrdtm.so && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5jf_prof_incr -o run --output-format csv -- python3 bench.py --workload incr --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off > gpurun_out/r5jf_prof_incr.log 2>&1
