# LDS-private row counts via bench args: configs[1] HS nodes (default 64; the
# LDS budget fits ~95 next to 64 context rows) and configs[4] (8 slots: private
# rows + staged atomic rows), alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r02z_priv
for rep in 1 2; do
  for spec in "c2 -1" "c2 96" "c5 -1" "c5 8" "c5 6"; do
    set -- $spec
    out=gpurun_out/r02z_priv/$1_pr$2_$rep
    timeout -k 10 200 python bench.py --config $1 --steps 2 --warmup 1 --cpu-seconds 0 --private-rows $2 > $out.json 2> $out.err || { echo fail; tail -3 $out.err; exit 1; }
    echo "$1 private_rows=$2 $rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
  done
done
