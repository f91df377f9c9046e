# configs[4]: device-coherent (sc1) row count vs speed and the SN quality gates.
set -o pipefail
mkdir -p gpurun_out/snc
for n in default 2000 1000; do
  if [ $n = default ]; then E=""; else E="W2V_SN_COHERENT_ROWS=$n"; fi
  env $E timeout -k 10 200 python bench.py --config c5 --cpu-seconds 0 > gpurun_out/snc/c5_$n.json 2> gpurun_out/snc/c5_$n.err || exit 1
  echo "coherent=$n $(python -c "import json;d=json.load(open('gpurun_out/snc/c5_$n.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['config']['env_knobs'])")"
  env $E timeout -k 10 300 python -u -m pytest tests/test_gpu_quality.py -q -s --timeout 250 --timeout-method thread -k shared_negatives > gpurun_out/snc/q_$n.log 2>&1
  echo "  quality rc=$? $(tail -1 gpurun_out/snc/q_$n.log)"
done
