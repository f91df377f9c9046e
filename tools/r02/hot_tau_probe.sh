# Automatic hot rows threshold (expected updates in flight of a W / C row;
# default 1) on the SG-NS presets: how much of the time the atomic rows cost.
set -o pipefail
mkdir -p gpurun_out/r02z_tau
for c in c3 c1; do
  for tau in 1 2 4; do
    out=gpurun_out/r02z_tau/${c}_tau$tau
    timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 --hot-auto $tau 1 > $out.json 2> $out.err || { echo fail; tail -3 $out.err; exit 1; }
    echo "$c hot_tau_rows=$tau $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
  done
done
