#!/bin/bash
# Instruction mix and wave-state cycles of one bench workload's kernels (two
# SQ counter passes of at most 8 SQ counters each, kernel trace off), summed
# per kernel by tools/pmc_summary.py:
#   tools/gpu_sq.sh <tag> <workload>
set -o pipefail
export TMPDIR=/tmp
R=$1; W=$2
O=gpurun_out
mkdir -p $O
B="python3 bench.py --workload $W --steps 2 --warmup 1 --cpu-sample 0 --pmc off"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU \
  -d $O/${R}_sq1_$W -o run --output-format csv -- $B > $O/${R}_sq1_$W.log 2>&1 || { echo "FAIL sq1"; tail -5 $O/${R}_sq1_$W.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAVES \
  -d $O/${R}_sq2_$W -o run --output-format csv -- $B > $O/${R}_sq2_$W.log 2>&1 || { echo "FAIL sq2"; tail -5 $O/${R}_sq2_$W.log; exit 1; }
python3 tools/pmc_summary.py $O/${R}_sq1_$W $O/${R}_sq2_$W > $O/${R}_${W}_sq_summary.txt
head -8 $O/${R}_${W}_sq_summary.txt
