#!/bin/bash
# round 5: host-side HIP API time of the incremental flat batches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/r5ht -o run --output-format csv -- python3 bench.py --workload incr --steps 1 --warmup 1 --cpu-sample 0 --pmc off > gpurun_out/r5ht.log 2>&1
