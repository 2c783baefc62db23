#!/bin/bash
# round 5: -structurizecfg-skip-uniform-regions per translation unit (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_ab.sh r5l "" "" cfg2 new lib:abtest/supdr/libcrdtm.so lib:abtest/suall/libcrdtm.so || exit 1
tools/gpu_ab.sh r5l "" "" incr_cfg2 new lib:abtest/suilr/libcrdtm.so lib:abtest/suall/libcrdtm.so || exit 1
tools/gpu_ab.sh r5l "" "" flat10m new lib:abtest/suall/libcrdtm.so || exit 1
tools/gpu_ab.sh r5l "" "" deep10m new lib:abtest/suall/libcrdtm.so || exit 1
tools/gpu_ab.sh r5l "" "" incr new lib:abtest/suall/libcrdtm.so
