#!/bin/bash
set -o pipefail
for mode in sg_hs cbow_hs; do for f in 16 64; do
  W2V_FLUSH_EVERY=$f W2V_PRIV_AVG=8 timeout -k 10 300 python bench.py --mode $mode --steps 1 --warmup 1 --cpu-seconds 0 --max-waves 1048576 > gpurun_out/hs.json 2> gpurun_out/hs.err || { tail -5 gpurun_out/hs.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/hs.json').read().strip().splitlines()[-1]); print(sys.argv[1],'F',sys.argv[2], round(d['value']/1e6,2), 'Mw/s frac', d['roofline']['frac'])" $mode $f
done; done
