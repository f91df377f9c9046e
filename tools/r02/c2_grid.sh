# configs[1] CBOW-HS: throughput over flush intervals x automatic hot-node
# threshold, then the paired quality probe for the candidate policies.
set -o pipefail
mkdir -p gpurun_out/c2g
for f in "64 32" "256 128" "512 256"; do
  set -- $f
  for tn in 1 2 4; do
    tag=f$1_c$2_tn$tn
    timeout -k 10 120 python bench.py --config c2 --steps 3 --warmup 1 --cpu-seconds 0 --flush-centers $1 --context-flush $2 --hot-auto 1 $tn > gpurun_out/c2g/$tag.json 2> gpurun_out/c2g/$tag.err || exit 1
    echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/c2g/$tag.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['config']['policy_used'])")"
  done
done
P="-;flush_centers=256,context_flush=128;flush_centers=256,context_flush=128,hot_tau_nodes=2;flush_centers=512,context_flush=256;flush_centers=512,context_flush=256,hot_tau_nodes=2"
for corpus in text8_like planted; do
  timeout -k 10 400 python -u tests/probes/quality_paired_probe.py $corpus cbow_hs 1,2,3 0 "$P" || exit 1
done
