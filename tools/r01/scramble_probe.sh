#!/bin/bash
# Contention probe: bench throughput per update policy, contiguous vs scrambled rows.
set -o pipefail
for lib in "" "word2vec_amd/lib_scr/libw2v_hip.so"; do
  for hp in "-1 0" "0 0" "10000 0"; do
    set -- $hp
    W2V_DEV_LIB=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 \
      --hot-rows $1 --private-rows $2 > gpurun_out/pb.json 2> gpurun_out/pb.err || { tail -5 gpurun_out/pb.err; exit 1; }
    python3 - "$lib" "$1" "$2" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/pb.json").read().strip().splitlines()[-1])
print(json.dumps({"lib": sys.argv[1] or "default", "hot": sys.argv[2], "priv": sys.argv[3],
                  "value": round(d["value"] / 1e6, 2), "frac": d["roofline"]["frac"]}))
PY
  done
done
