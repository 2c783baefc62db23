set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --cpu-sample 0 > gpurun_out/r4p_flat10m.log 2>&1 || { tail -20 gpurun_out/r4p_flat10m.log; exit 1; }
timeout -k 10 400 python -u bench.py --workload incr --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/r4p_incr.log 2>&1 || { tail -20 gpurun_out/r4p_incr.log; exit 1; }
timeout -k 10 400 python -u bench.py --workload trees --cpu-sample 0 --steps 3 --warmup 1 > gpurun_out/r4p_trees.log 2>&1 || { tail -20 gpurun_out/r4p_trees.log; exit 1; }
echo done
