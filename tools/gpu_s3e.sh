set -e
export TMPDIR=/tmp
O=gpurun_out/s3e
mkdir -p $O
for g in 512 1024 2048; do
  for w in flat10m deep10m; do
    CRDTM_PRE_GRID=$g timeout -k 10 300 python -u bench.py --workload $w --cpu-sample 0 --steps 20 > $O/bench_${w}_$g.log 2>&1
  done
done
