# Round 3, lease r: configs[4] LDS-private C rows — throughput and quality at d512 / neg 15.
set -o pipefail
TAG=${1:-r03r}
mkdir -p gpurun_out/$TAG
for pr in -1 0 2 4 -1 0; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --private-rows $pr > gpurun_out/$TAG/c5_pr$pr.json 2> gpurun_out/$TAG/c5_pr$pr.err || exit 1
  echo "c5 private_rows=$pr $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_pr$pr.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
done
timeout -k 10 400 python -u tools/r03/c5_hot_probe.py -2 11,12,13 0 0 0,2,4 8 > gpurun_out/$TAG/c5_priv.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_priv.log
timeout -k 10 400 python -u tools/r03/c5_hot_probe.py -2 11,12,13 0 0 -1 8 64,256 > gpurun_out/$TAG/c5_flush.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_flush.log
for fl in 64 256; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --flush-centers $fl > gpurun_out/$TAG/c5_fl$fl.json 2> gpurun_out/$TAG/c5_fl$fl.err || exit 1
  echo "c5 flush=$fl $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_fl$fl.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
done
echo PHASE_DONE
