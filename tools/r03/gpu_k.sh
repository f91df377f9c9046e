# Round 3, lease k: saturation exchange exactness; R = 8 studies (50 M and 400 M
# tokens); configs[0] with paired contexts at d100 (variant pair2).
set -o pipefail
TAG=${1:-r03k}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_replicas.py -m gpu -x -v -k "exchange" --timeout 200 --timeout-method thread > gpurun_out/$TAG/replica_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/$TAG/replica_tests.log | tail -6; [ $rc -eq 0 ] || exit 1
bash tools/r03/ab.sh $TAG pair2 "c1" 2 || exit 1
timeout -k 10 600 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8 --rounds 64,256 --gmodes sat0.002,sat0.0005 > gpurun_out/$TAG/replicas_sat.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/replicas_sat.log
timeout -k 10 900 python -u tools/r03/replica_study.py --tokens 400000000 --planted-frac 0.006 --replicas 8 --rounds 4,16,64 --gmodes average,sat0.002,sum > gpurun_out/$TAG/big.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/big.log
echo PHASE_DONE
