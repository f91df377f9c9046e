#!/bin/bash
set -o pipefail
for mode in sg_hs cbow_hs; do for w in 128 256 512 1024; do
  timeout -k 10 300 python bench.py --mode $mode --steps 1 --warmup 1 --cpu-seconds 0 --max-waves $w > gpurun_out/hs.json 2> gpurun_out/hs.err || { tail -5 gpurun_out/hs.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/hs.json').read().strip().splitlines()[-1]); print(sys.argv[1],'waves',sys.argv[2], round(d['value']/1e6,2), 'Mw/s frac', d['roofline']['frac'])" $mode $w
done; done
