#!/bin/bash
# tests (a pytest -k filter, or "" for none) on the in-tree build, then an A/B of bench lines:
#   tools/gpu_ab.sh <tag> "<pytest files>" "<-k expr>" <workload> <variant> [variant ...]
# variant: new (in-tree build), lib:<path>, ab:<CRDTM_AB value>, env:VAR=value
set -o pipefail
T=$1; F=$2; K=$3; W=$4; shift 4
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$F" ]; then
  timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${T}_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    envs=""; name=new
    if [[ $v == lib:* ]]; then envs="CRDTM_LIB=${v#lib:}"; name=$(echo ${v#lib:} | tr '/' '_');
    elif [[ $v == ab:* ]]; then envs="CRDTM_AB=${v#ab:}"; name=ab_${v#ab:};
    elif [[ $v == env:* ]]; then envs="${v#env:}"; name=$(echo ${v#env:} | tr '=/ ' '___'); fi
    f=gpurun_out/${T}_${W}_${name}_$rep.log
    env $envs timeout -k 10 300 python -u bench.py --workload $W --steps ${STEPS:-10} --cpu-sample 0 --pmc off --verbose > $f 2>&1 || { echo FAIL $v; tail -5 $f; exit 1; }
    echo "$name $rep $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"
  done
done
