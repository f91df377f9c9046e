# One bench line per BASELINE.json config preset (bench.py --config cN) on one
# GPU. usage (GPU box): bash tools/bench_configs.sh
set -o pipefail
mkdir -p gpurun_out
for c in c1 c2 c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-seconds ${CPU_SECONDS:-6} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -5 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));r=d['roofline'];print('$c', d['config']['workload'][:60], round(d['value']/1e6,1), 'M words/s frac', r['frac'], 'cpu', (d['cpu_baseline'] or {}).get('value'))"
done
