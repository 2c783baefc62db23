set -e
export TMPDIR=/tmp
O=gpurun_out/s3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize_parity.py -m gpu -x -v -k "interleaved or forced" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload deep10m_il --cpu-sample 0 > $O/bench_deep10m_il.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg2 --force-replay --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 > $O/bench_cfg2_forced.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_deep10m_il -o run --output-format csv -- python3 bench.py --workload deep10m_il --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 > $O/prof_deep10m_il.log 2>&1
