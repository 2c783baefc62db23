set -e
export TMPDIR=/tmp
O=gpurun_out/s3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for w in flat10m deep10m; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-sample 0 > $O/bench_$w.log 2>&1
done
bash tools/profile_workload.sh s3c flat10m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_deep10m -o run --output-format csv -- python3 bench.py --workload deep10m --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 > $O/prof_deep10m.log 2>&1
