# Round 3, lease f: replica tests (hot-row exchange, split), then the
# 8-replica study with frequent hot-row exchanges between full ones.
set -o pipefail
TAG=${1:-r03f}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/replica_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/$TAG/replica_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
S="timeout -k 10 500 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8"
$S --rounds 512 --gmodes adaptive,split1000 > gpurun_out/$TAG/full512.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/full512.log
for K in 4096 32768; do
  $S --rounds 8 --hot-rows $K --hot-rounds 512 --gmodes adaptive,sum,split1000,average > gpurun_out/$TAG/hot$K.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/$TAG/hot$K.log | tail -4
done
