set -e
export TMPDIR=/tmp
O=gpurun_out/s3g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_incremental.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload incr --cpu-sample 0 > $O/bench_incr.log 2>&1
