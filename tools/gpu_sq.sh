#!/bin/bash
# SQ instruction counters of one workload's kernels (one rocprofv3 --pmc pass):
#   tools/gpu_sq.sh <tag> <workload> <kernel-substring>
set -euo pipefail
export TMPDIR=/tmp
T=$1; W=$2; K=$3
O=gpurun_out
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d $O/${T}_sq_$W -o run --output-format csv -- python3 bench.py --workload $W --steps 1 --warmup 0 --profile-steps 1 --cpu-sample 0 --pmc off > $O/${T}_sq_$W.log 2>&1
python3 tools/sq_summary.py $O/${T}_sq_$W $K > $O/${T}_${W}_sq_summary.txt
