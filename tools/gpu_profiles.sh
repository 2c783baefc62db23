#!/bin/bash
# Refreshes every workload's bench line (default steps, CPU baseline on this
# host), rocprofv3 kernel stats and FETCH/WRITE PMC summaries on the GPU box:
#   tools/gpu_profiles.sh <tag> [workload ...]
# Outputs gpurun_out/<tag>_<w>_{bench.log,kernel_stats.csv,pmc.json,pmc_summary.txt}
set -euo pipefail
export TMPDIR=/tmp
T=$1; shift
WS=${*:-flat10m deep10m cfg2 trees cfg1 incr}
O=gpurun_out
mkdir -p $O
for w in $WS; do
  timeout -k 10 400 python3 -u bench.py --workload $w > $O/${T}_${w}_bench.log 2>&1
  if [ "$w" != cfg1 ] && [ "$w" != incr ]; then
    bash tools/profile_workload.sh $T $w
    cp $O/${T}_prof_$w.log $O/${T}_${w}_prof_bench.log
  fi
done
