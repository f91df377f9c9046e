set -o pipefail
mkdir -p gpurun_out/r02z_c2ctx
for rep in 1 2; do
  for cf in 0 256; do
    out=gpurun_out/r02z_c2ctx/c2_cf${cf}_$rep
    timeout -k 10 150 python bench.py --config c2 --steps 3 --warmup 1 --cpu-seconds 0 --context-flush $cf > $out.json 2> $out.err || { echo fail; exit 1; }
    echo "c2 context_flush=$cf $rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
  done
done
