#!/bin/bash
# ILR: incremental tests, then one debug pass of incr_cfg2 (per-batch decisions), then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ilr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ilr_tests.log; [ $rc = 0 ] || exit $rc
CRDTM_ILR_DEBUG=1 timeout -k 10 300 python -u bench.py --workload incr_cfg2 --steps 1 --warmup 0 --pmc off --cpu-sample 0 > gpurun_out/ilr_dbg.log 2>&1 || { tail -20 gpurun_out/ilr_dbg.log; exit 1; }
grep "^ilr:" gpurun_out/ilr_dbg.log | sort | uniq -c | sort -rn | head -20
timeout -k 10 300 python -u bench.py --workload incr_cfg2 --cpu-sample 0 --pmc off --verbose > gpurun_out/ilr_bench.log 2>&1 || { tail -20 gpurun_out/ilr_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"batches_remerged": [0-9]*\|"paths": {[^}]*}' gpurun_out/ilr_bench.log
