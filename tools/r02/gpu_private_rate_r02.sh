#!/bin/bash
# Round-2 sweep of the private-row rate threshold (w2v_dev_set_private_rate):
# paired quality on the three corpora and throughput on the presets.
set -o pipefail
TAG=${1:-r02r}
mkdir -p gpurun_out
P="-;private_rate=0.05;private_rate=0.1;private_rate=0.2;private_rate=0.5"
for c in text8_small planted text8_like; do
  seeds=1; [ $c = planted ] && seeds=1,2
  timeout -k 10 400 python -u tests/probes/quality_paired_probe.py $c sg_ns,cbow_hs $seeds 0 "$P" > gpurun_out/${TAG}_$c.log 2>&1 || { echo "probe $c failed"; tail -3 gpurun_out/${TAG}_$c.log; }
  cut -c1-60,100-230 gpurun_out/${TAG}_$c.log | grep corpus
done
for c in c3 c1 c2; do
  for mu in 0 0.1 0.2; do
    timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 0 --private-rate $mu > gpurun_out/${TAG}_bench_${c}_$mu.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,2), 'M words/s', d['roofline']['frac'], d['config']['policy_used'])" gpurun_out/${TAG}_bench_${c}_$mu.json $c $mu
  done
done
