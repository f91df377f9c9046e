# Round 3, lease j: 8 replicas on a large corpus (400 M tokens), rounds that
# fill the chip (3-12 M tokens per replica per round): which exchange holds quality?
set -o pipefail
TAG=${1:-r03j}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u tools/r03/replica_study.py --tokens 400000000 --planted-frac 0.006 --replicas 8 --rounds 4,16,64 --gmodes average,sat0.002,sum > gpurun_out/$TAG/big.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/big.log
echo PHASE_DONE
