set -e
export TMPDIR=/tmp
O=gpurun_out/s3j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize_parity.py -m gpu -x -v -k "incremental_flat_1m or forced" --timeout 170 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload deep10m --cpu-sample 0 > $O/bench_deep10m.log 2>&1
