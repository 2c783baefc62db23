set -e
export TMPDIR=/tmp
O=gpurun_out/s3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize_parity.py -m gpu -x -v -k "forced" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg2 --force-replay --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 > $O/bench_cfg2_forced.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d $O/sq_trees -o run --output-format csv -- python3 bench.py --workload trees --steps 1 --warmup 0 --profile-steps 1 --cpu-sample 0 > $O/sq_trees.log 2>&1
python3 tools/sq_summary.py $O/sq_trees forest > $O/sq_trees_summary.txt
