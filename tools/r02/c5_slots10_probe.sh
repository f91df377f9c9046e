# configs[4] with 10 LDS row slots (single transpose buffer): private rows 8
# (default) / 10 / 4, alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r02z_c5s10
for rep in 1 2; do
  for pr in -1 10 4; do
    out=gpurun_out/r02z_c5s10/c5_pr${pr}_$rep
    timeout -k 10 200 python bench.py --config c5 --steps 2 --warmup 1 --cpu-seconds 0 --private-rows $pr > $out.json 2> $out.err || { echo fail; tail -3 $out.err; exit 1; }
    echo "c5 private_rows=$pr $rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
  done
done
