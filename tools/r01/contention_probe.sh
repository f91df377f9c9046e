#!/bin/bash
# Atomic-policy slowdown: per-row contention (Zipf) or per-step atomic latency (uniform corpus too)?
set -o pipefail
run() {  # zipf_s hot priv
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --zipf-s $1 --hot-rows $2 --private-rows $3 \
    > gpurun_out/cp.json 2> gpurun_out/cp.err || { tail -5 gpurun_out/cp.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/cp.json').read().strip().splitlines()[-1]); print('s',sys.argv[1],'hot',sys.argv[2],'priv',sys.argv[3], round(d['value']/1e6,2), 'Mw/s frac', d['roofline']['frac'])" $1 $2 $3
}
run 0 0 0 && run 0 -1 0 && run 1 10 0 && run 1 100 0 && run 1 1000 0 && run 0.5 -1 0 && run 0.5 0 0
