# CBOW-HS (c2): throughput and planted-corpus quality vs the atomic-row threshold.
# usage (GPU box): bash tools/hs_hot_rows.sh
set -o pipefail
mkdir -p gpurun_out
for H in 250 500 1000 2000; do
  timeout -k 10 200 python -u bench.py --config c2 --cpu-seconds 0 --hot-rows $H > gpurun_out/hh_$H.json 2> gpurun_out/hh_$H.err || { tail -5 gpurun_out/hh_$H.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/hh_$H.json'));print('c2 hot_rows $H', round(d['value']/1e6,2), 'M words/s')"
done | tee gpurun_out/hs_hot_rows.log
timeout -k 10 400 python -u tools/quality_policy.py cbow_hs policy=default policy=hot_rows=250 policy=hot_rows=500 policy=hot_rows=2000 2>&1 | tee -a gpurun_out/hs_hot_rows.log
