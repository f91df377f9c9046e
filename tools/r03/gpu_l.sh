# Round 3, lease l: 8 replicas with 8x the data (400 M tokens, planted 0.05),
# and 8 replicas at the same total concurrency as one (max_waves 512 = 64 each).
set -o pipefail
TAG=${1:-r03l}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u tools/r03/replica_study.py --tokens 400000000 --planted-frac 0.05 --replicas 8 --rounds 4,16,64 --gmodes average,sat0.002 > gpurun_out/$TAG/big.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/big.log
timeout -k 10 600 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8 --max-waves 512 --rounds 256 --gmodes sat0.002,sum > gpurun_out/$TAG/w512.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/w512.log
echo PHASE_DONE
