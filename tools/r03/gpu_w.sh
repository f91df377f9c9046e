# Round 3, lease w: the hot-row threshold at the headline's scale, 3 seeds.
set -o pipefail
TAG=${1:-r03w}
mkdir -p gpurun_out/$TAG
for tau in 1 2 4 16; do
  timeout -k 10 300 python -u tools/r03/replica_study.py --tokens 50000000 --filler 1000000 --dim 300 --planted-frac 0.05 --replicas "" --hot-tau $tau --seeds 1,2,3 > gpurun_out/$TAG/quality_tau$tau.log 2>&1 || exit 1
  echo "tau $tau: $(grep '"R": 1' gpurun_out/$TAG/quality_tau$tau.log | python -c "import sys,json;r=[json.loads(l) for l in sys.stdin];print([(x['analogy'],x['similarity']) for x in r], 'mean', round(sum(x['analogy'] for x in r)/len(r),2), round(sum(x['similarity'] for x in r)/len(r),2))")"
done
for tau in 1 2 1 2; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --hot-auto $tau 1 > gpurun_out/$TAG/c3_tau$tau.json 2> gpurun_out/$TAG/c3_tau$tau.err || exit 1
  echo "c3 tau=$tau $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c3_tau$tau.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used']['hot_rows'])")"
done
echo PHASE_DONE
