#!/bin/bash
# A/B on one box: bench.py once per variant, interleaved, 2 rounds.
# A variant is a CRDTM_AB value ("" = default) or lib:<path> (CRDTM_LIB).
#   tools/ab_bench.sh <tag> <workload> <variant> [variant ...]
set -o pipefail
T=$1; W=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    if [[ $v == lib:* ]]; then envs="CRDTM_LIB=${v#lib:}"; name=$(echo ${v#lib:} | tr '/' '_'); else envs="CRDTM_AB=$v"; name=${v:-base}; fi
    f=gpurun_out/${T}_${W}_${name}_$rep.log
    env $envs timeout -k 10 300 python -u bench.py --workload $W --cpu-sample 0 --pmc off --verbose > $f 2>&1 || { echo FAIL $v; tail -5 $f; exit 1; }
    echo "$name $rep $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) | $(grep -E '^  k_' $f | head -6 | awk '{print $1, $2}' | tr '\n' ' ')"
  done
done
