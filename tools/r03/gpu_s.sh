# Round 3, lease s: configs[4] — can 10 LDS-private rows with a shorter flush
# interval keep both the negative-15 quality gate and their throughput?
set -o pipefail
TAG=${1:-r03s}
mkdir -p gpurun_out/$TAG
for fl in 256 128 64; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --private-rows 10 --flush-centers $fl > gpurun_out/$TAG/c5_fl$fl.json 2> gpurun_out/$TAG/c5_fl$fl.err || exit 1
  echo "c5 private_rows=10 flush=$fl $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_fl$fl.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
done
timeout -k 10 400 python -u tools/r03/c5_hot_probe.py -2 11,12,13 0 0 10 8 256,128,64 > gpurun_out/$TAG/c5_flush.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_flush.log
echo PHASE_DONE
