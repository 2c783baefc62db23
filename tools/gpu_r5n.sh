#!/bin/bash
# round 5: kernel traces of the incremental workloads and flat10m (timelines)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in incr_cfg2 incr flat10m; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5n_prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off > gpurun_out/r5n_prof_$w.log 2>&1 || { echo FAIL $w; tail -5 gpurun_out/r5n_prof_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5n_prof_$w.log | head -1)"
done
