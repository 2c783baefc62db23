#!/bin/bash
# A round's judged evidence for some workloads, on the GPU box (through gpurun):
#   tools/gpu_profiles.sh <round tag> <workload> [workload ...]
# per workload: the default bench line (live PMC traffic, CPU baseline) in
# gpurun_out/<tag>_<w>_bench.log, then tools/profile_workload.sh (kernel trace
# and stats, FETCH_SIZE / WRITE_SIZE passes, the per-kernel PMC summary) and
# the last step's timeline (tools/timeline.py). Copy what is judged into
# profiles/ afterwards.
set -o pipefail
export TMPDIR=/tmp
R=$1; shift
O=gpurun_out
mkdir -p $O
for w in "$@"; do
  timeout -k 10 400 python3 -u bench.py --workload $w > $O/${R}_${w}_bench.log 2>&1 || { echo "FAIL bench $w"; tail -5 $O/${R}_${w}_bench.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/${R}_${w}_bench.log | head -1)"
  bash tools/profile_workload.sh $R $w || { echo "FAIL profile $w"; exit 1; }
  # (a step of the single-document workloads starts at the tree reset, whose
  # launch also initialises the result block; the others at the result init)
  case $w in flat10m|deep10m|deep10m_il|cfg1|cfg2) m=k_reset_root ;; *) m=k_dres_init ;; esac
  python3 tools/timeline.py $O/${R}_prof_$w/run_kernel_trace.csv $m -2 > $O/${R}_${w}_timeline.txt 2>&1 || true
  tail -1 $O/${R}_${w}_timeline.txt
done
