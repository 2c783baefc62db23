#!/bin/bash
# SQ counters of the forest replay kernels (default: one wave per document)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/sqf_$1 -o run --output-format csv -- python3 bench.py --workload trees --steps 1 --warmup 0 --profile-steps 1 --cpu-sample 0 > $O/sqf_$1.log 2>&1
  python3 tools/sq_summary.py $O/sqf_$1 forest > $O/sqf_$1.txt
}
run ${1:-wave}
