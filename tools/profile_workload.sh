#!/bin/bash
# Profiles one bench workload on the GPU box (run through gpurun):
#   tools/profile_workload.sh <workload> [extra bench args]
# Writes gpurun_out/prof_<w>/ (kernel trace + stats), gpurun_out/pmc_<w>_{fetch,write}/
# (one counter per pass, as MI355X_MICROARCH.md prescribes) and the bench line.
set -euo pipefail
export TMPDIR=/tmp
W=$1; shift
B="python3 bench.py --workload $W --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 $*"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$W -o run --output-format csv -- $B > gpurun_out/prof_$W.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${W}_fetch -o run --output-format csv -- $B > gpurun_out/pmc_${W}_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${W}_write -o run --output-format csv -- $B > gpurun_out/pmc_${W}_write.log 2>&1
