# Round 3, lease a: the vocab-aware hot-row threshold (auto vs the old tau 1) on
# the per-pair presets, its paired text8-like quality, then the GPU suite.
set -o pipefail
TAG=${1:-r03a}
mkdir -p gpurun_out/$TAG
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
for rep in 1 2; do
  for c in c3 c1 c2; do
    for tau in 0 1; do
      out=gpurun_out/$TAG/${c}_tau${tau}_$rep
      timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 --hot-auto $tau 1 > $out.json 2> $out.err || stop "bench $c tau$tau" $?
      echo "$c tau=$tau rep=$rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
    done
  done
done
timeout -k 10 600 python -u tests/probes/quality_paired_probe.py text8_like sg_ns,cbow_hs 1,2,3 0 "-;hot_tau_rows=1" > gpurun_out/$TAG/quality_text8_like.log 2>&1 || stop quality $?
cat gpurun_out/$TAG/quality_text8_like.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 || stop gpu_tests $?
tail -3 gpurun_out/$TAG/gpu_tests.log
