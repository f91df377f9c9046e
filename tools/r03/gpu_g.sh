# Round 3, lease g: configs[4] atomic rows (throughput and quality at d512 / neg 15).
set -o pipefail
TAG=${1:-r03g}
mkdir -p gpurun_out/$TAG
for h in -2 500 250 100; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --hot-rows $h > gpurun_out/$TAG/c5_hot$h.json 2> gpurun_out/$TAG/c5_hot$h.err || exit 1
  echo "c5 hot_rows=$h $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_hot$h.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
done
timeout -k 10 600 python -u tools/r03/c5_hot_probe.py -2,500,250,100 > gpurun_out/$TAG/c5_quality.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_quality.log
