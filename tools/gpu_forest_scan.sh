set -o pipefail
mkdir -p gpurun_out
for d in 4096 8192 10240 12500 16384; do
  timeout -k 10 200 python -u bench.py --workload trees --docs-per-gpu $d --cpu-sample 0 --pmc off --verbose > gpurun_out/r6x_trees_$d.log 2>&1 || { echo FAIL $d; tail -5 gpurun_out/r6x_trees_$d.log; exit 1; }
  echo "$d $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6x_trees_$d.log | head -1) $(grep -E 'k_forest_wave' gpurun_out/r6x_trees_$d.log | head -1)"
done
