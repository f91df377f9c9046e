set -o pipefail
mkdir -p gpurun_out/c2p
for v in "def:" "f128:--flush-centers 128" "cf64:--context-flush 64" "both:--flush-centers 128 --context-flush 64" "f256:--flush-centers 256 --context-flush 128"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 120 python bench.py --config c2 --steps 3 --warmup 1 --cpu-seconds 0 $args > gpurun_out/c2p/$tag.json 2> gpurun_out/c2p/$tag.err || exit 1
  echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/c2p/$tag.json'));print(round(d['value']/1e6,2),d['roofline']['frac'])")"
done
PASSES=atom timeout -k 10 200 bash tools/pmc.sh c2atom --config c2
