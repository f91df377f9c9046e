# Round 3, lease n: 8 averaged replicas with the learning rate scaled by R
# (the linear scaling rule of large-batch SGD) at chip-filling cadences.
set -o pipefail
TAG=${1:-r03n}
mkdir -p gpurun_out/$TAG
for f in 0.02 0.015; do
  for lr in 8 4; do
    timeout -k 10 400 python -u tools/r03/replica_study.py --tokens 400000000 --planted-frac $f --replicas 8 --rounds 1,4,16 --gmodes average --lr-scale $lr > gpurun_out/$TAG/big_f${f}_lr$lr.log 2>&1 || exit 1
    grep -v amdgpu.ids gpurun_out/$TAG/big_f${f}_lr$lr.log
  done
done
timeout -k 10 400 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8 --rounds 4,16,64 --gmodes average --lr-scale 8 > gpurun_out/$TAG/f0.05_lr8.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/f0.05_lr8.log
echo PHASE_DONE
