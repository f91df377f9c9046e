#!/bin/bash
# bench throughput per update policy: "hot priv extra-env" triples
set -o pipefail
while read -r hot priv env; do
  [ -z "$hot" ] && continue
  env $env timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --hot-rows $hot --private-rows $priv \
    > gpurun_out/pol.json 2> gpurun_out/pol.err || { tail -5 gpurun_out/pol.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/pol.json').read().strip().splitlines()[-1]); print('hot',sys.argv[1],'priv',sys.argv[2],sys.argv[3], round(d['value']/1e6,2), 'Mw/s frac', d['roofline']['frac'])" "$hot" "$priv" "$env"
done
