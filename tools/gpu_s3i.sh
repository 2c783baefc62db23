set -e
export TMPDIR=/tmp
O=gpurun_out/s3i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 -u bench.py --workload incr > gpurun_out/r2_incr_bench.log 2>&1
timeout -k 10 300 python3 -u bench.py > $O/bench_flat10m.log 2>&1
