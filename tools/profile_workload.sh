#!/bin/bash
# Profiles one bench workload on the GPU box (run through gpurun):
#   tools/profile_workload.sh <round> <workload> [extra bench args]
# Writes gpurun_out/<round>_prof_<w>/ (kernel trace + stats),
# gpurun_out/<round>_pmc_<w>_{fetch,write}/ (one counter per pass, as
# MI355X_MICROARCH.md prescribes), the bench lines and the per-kernel PMC
# summary gpurun_out/<round>_<w>_pmc{.json,_summary.txt}.
set -euo pipefail
export TMPDIR=/tmp
R=$1; W=$2; shift 2
B="python3 bench.py --workload $W --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 --pmc off $*"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${R}_prof_$W -o run --output-format csv -- $B > $O/${R}_prof_$W.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/${R}_pmc_${W}_fetch -o run --output-format csv -- $B > $O/${R}_pmc_${W}_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/${R}_pmc_${W}_write -o run --output-format csv -- $B > $O/${R}_pmc_${W}_write.log 2>&1
python3 tools/pmc_summary.py $O/${R}_pmc_${W}_fetch $O/${R}_pmc_${W}_write --json $O/${R}_${W}_pmc.json > $O/${R}_${W}_pmc_summary.txt
cp $O/${R}_prof_$W/run_kernel_stats.csv $O/${R}_${W}_kernel_stats.csv
