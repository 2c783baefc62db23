#!/bin/bash
# Kernel-trace timeline of one bench workload (no counters): a short bench
# under rocprofv3 --kernel-trace, then tools/timeline.py on the last complete
# step. Extra env (A/B switches) is passed through.
#   tools/gpu_trace.sh <tag> <workload> [marker]
set -euo pipefail
export TMPDIR=/tmp
T=$1; W=$2; M=${3:-k_dres_init}
O=gpurun_out
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/${T}_trace_$W -o run --output-format csv -- \
  python3 bench.py --workload $W --steps 4 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off > $O/${T}_trace_$W.log 2>&1
python3 tools/timeline.py $O/${T}_trace_$W/run_kernel_trace.csv $M -3 > $O/${T}_${W}_timeline.txt
cat $O/${T}_${W}_timeline.txt
