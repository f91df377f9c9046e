#!/bin/bash
# Round-2 update-policy sweep (automatic hot rows): per-preset bench lines with
# the automatic rule and the previous fixed 1000 rows, then paired quality.
# usage (GPU box): bash tools/gpu_policy_r02.sh <tag>
set -o pipefail
TAG=${1:-r02b}
mkdir -p gpurun_out
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
for c in c3 c2 c1 c5; do
  for hr in -2 1000; do
    timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 0 --hot-rows $hr > gpurun_out/${TAG}_bench_${c}_hot${hr}.json 2> gpurun_out/${TAG}_bench_${c}_hot${hr}.err || stop "bench $c $hr" $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,2), 'M words/s', d['roofline']['frac'], d['config']['policy_used'])" gpurun_out/${TAG}_bench_${c}_hot${hr}.json $c $hr
  done
done
timeout -k 10 600 python -u tests/probes/quality_paired_probe.py text8_like cbow_hs,sg_ns 1,2,3 0 "-;hot_auto=0.5;hot_auto=2;hot_rows=1000" > gpurun_out/${TAG}_probe_text8.log 2>&1 || stop probe $?
cat gpurun_out/${TAG}_probe_text8.log
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py planted sg_ns,sg_hs,cbow_ns,cbow_hs 1,2,3 0 "-;hot_rows=1000" > gpurun_out/${TAG}_probe_planted.log 2>&1 || stop probe2 $?
cat gpurun_out/${TAG}_probe_planted.log
echo PHASE_DONE
