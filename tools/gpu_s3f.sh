set -e
export TMPDIR=/tmp
O=gpurun_out/s3f
mkdir -p $O
timeout -k 10 300 python -u bench.py --workload cfg2 --cpu-sample 0 --steps 5 > $O/bench_cfg2_base.log 2>&1
CRDTM_PDR_LOG_MIN=1000000000 timeout -k 10 300 python -u bench.py --workload cfg2 --cpu-sample 0 --steps 5 > $O/bench_cfg2_nolog.log 2>&1
timeout -k 10 300 python -u bench.py --workload flat10m --cpu-sample 0 > $O/bench_flat10m.log 2>&1
