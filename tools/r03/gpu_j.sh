# Round 3, lease j: is the R = 8 quality loss the exchange or the in-launch
# concurrency? Same total waves for R = 1 and R = 8 (each replica max_waves/8).
set -o pipefail
TAG=${1:-r03j}
mkdir -p gpurun_out/$TAG
S="timeout -k 10 600 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8"
$S --max-waves 512 --rounds 64,256 --gmodes sum,adaptive,average > gpurun_out/$TAG/w512.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/w512.log
$S --max-waves 64 --rounds 256 --gmodes sum,adaptive > gpurun_out/$TAG/w64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/w64.log
echo PHASE_DONE
