#!/bin/bash
# Round-2 follow-up: separate thresholds for W / C rows and Huffman nodes.
set -o pipefail
TAG=${1:-r02c}
mkdir -p gpurun_out
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
for c in c3 c1 c2; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 0 > gpurun_out/${TAG}_bench_${c}.json 2> gpurun_out/${TAG}_bench_${c}.err || stop "bench $c" $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M words/s', d['roofline']['frac'], d['config']['policy_used'])" gpurun_out/${TAG}_bench_${c}.json $c
done
timeout -k 10 600 python -u tests/probes/quality_paired_probe.py text8_like cbow_hs,sg_ns 1,2,3 0 "-;hot_tau_rows=0.5" > gpurun_out/${TAG}_probe_text8.log 2>&1 || stop probe $?
cat gpurun_out/${TAG}_probe_text8.log
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py planted sg_ns,sg_hs,cbow_ns,cbow_hs 1,2,3 0 "-" > gpurun_out/${TAG}_probe_planted.log 2>&1 || stop probe2 $?
cat gpurun_out/${TAG}_probe_planted.log
echo PHASE_DONE
