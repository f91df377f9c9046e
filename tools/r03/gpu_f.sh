# Round 3, lease f: replica tests (hot-row exchange, split), then the
# 8-replica study with frequent hot-row exchanges between full ones.
set -o pipefail
TAG=${1:-r03f}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py -k "split or hot_rows or one_rank" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/replica_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/$TAG/replica_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
S="timeout -k 10 500 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8"
$S --rounds 512 --gmodes adaptive,split1000 > gpurun_out/$TAG/full512.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/full512.log
for K in 4096 32768; do
  $S --rounds 8 --hot-rows $K --hot-rounds 512 --gmodes adaptive,sum,split1000,average > gpurun_out/$TAG/hot$K.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/$TAG/hot$K.log | tail -4
done
# more LDS-private output rows on the SG-NS presets (fewer memory-side atomics)
for c in c3 c1; do
  for pr in -1 127; do
    timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 --private-rows $pr > gpurun_out/$TAG/${c}_pr$pr.json 2> gpurun_out/$TAG/${c}_pr$pr.err || exit 1
    echo "$c private_rows=$pr $(python -c "import json;d=json.load(open('gpurun_out/$TAG/${c}_pr$pr.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
  done
done
timeout -k 10 400 python -u tests/probes/quality_paired_probe.py text8_like sg_ns 1,2,3 0 "-;private_rows=127" > gpurun_out/$TAG/priv_quality.log 2>&1 || exit 1
cat gpurun_out/$TAG/priv_quality.log
