set -o pipefail
mkdir -p gpurun_out
for v in 0; do
CRDTM_FILL_SIDE=$v timeout -k 10 300 python -u bench.py --cpu-sample 0 --verbose > gpurun_out/r3c_fill$v.log 2>&1 || exit 1
echo "fill_side=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3c_fill$v.log | head -1)"
done
