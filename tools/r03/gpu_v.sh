# Round 3, lease v: the hot-row threshold at the headline's scale (d300, a
# 1M-rank planted Zipf corpus: rho = waves x (window + 1) / V ~ 0.1): quality
# of one replica at tau 1 / 4 / 8 / 16, and configs[2]'s throughput at each.
set -o pipefail
TAG=${1:-r03v}
mkdir -p gpurun_out/$TAG
for tau in 1 4 8 16; do
  timeout -k 10 300 python -u tools/r03/replica_study.py --tokens 50000000 --filler 1000000 --dim 300 --planted-frac 0.05 --replicas "" --hot-tau $tau > gpurun_out/$TAG/quality_tau$tau.log 2>&1 || exit 1
  echo "tau $tau: $(grep -v amdgpu.ids gpurun_out/$TAG/quality_tau$tau.log | tail -2 | tr '\n' ' ')"
done
for tau in 4 8 16 4 8 16; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --hot-auto $tau 1 > gpurun_out/$TAG/c3_tau$tau.json 2> gpurun_out/$TAG/c3_tau$tau.err || exit 1
  echo "c3 tau=$tau $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c3_tau$tau.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used']['hot_rows'])")"
done
echo PHASE_DONE
