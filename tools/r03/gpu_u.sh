# Round 3, lease u: configs[4] LDS-private rows flushed as a plain sum at short
# intervals (no averaging): quality at d512 / neg 15 and throughput.
set -o pipefail
TAG=${1:-r03u}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u tools/r03/c5_hot_probe.py -2 11,12,13 0 0 10 0 16,64 > gpurun_out/$TAG/c5_sum_flush.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_sum_flush.log
for fl in 16 64; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --private-rows 10 --private-average 0 --flush-centers $fl > gpurun_out/$TAG/c5_fl$fl.json 2> gpurun_out/$TAG/c5_fl$fl.err || exit 1
  echo "c5 private_rows=10 sum flush=$fl $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_fl$fl.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
done
timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/$TAG/c5_default.json 2> gpurun_out/$TAG/c5_default.err || exit 1
echo "c5 default $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_default.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
echo PHASE_DONE
