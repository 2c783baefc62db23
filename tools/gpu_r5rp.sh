#!/bin/bash
# round 5: the replica fold's output in the last k_rep_max workgroup, A/B on the general-path workloads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in deep10m deep10m_il incr; do tools/gpu_ab.sh r5rp "" "" $w new lib:abtest/prerep/libcrdtm.so || exit 1; done
