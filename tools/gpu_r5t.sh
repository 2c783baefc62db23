#!/bin/bash
# round 5: findInsertion's stop decided before the next word is read (forest, per-dict replays), tests + A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5t_tests.log; [ $rc = 0 ] || exit $rc
for w in trees cfg2 deep10m_il cfg1; do tools/gpu_ab.sh r5t "" "" $w new lib:abtest/prev/libcrdtm.so || exit 1; done
