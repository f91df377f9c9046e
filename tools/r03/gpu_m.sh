# Round 3, lease m: 8 replicas at bench.py's N>1 cadence on a 400 M-token corpus
# whose single-replica scores are below the metric's ceiling (planted 0.01-0.02).
set -o pipefail
TAG=${1:-r03m}
mkdir -p gpurun_out/$TAG
for f in 0.01 0.015 0.02; do
  timeout -k 10 400 python -u tools/r03/replica_study.py --tokens 400000000 --planted-frac $f --replicas 8 --rounds 1,4 --gmodes average,row_average,sum > gpurun_out/$TAG/big_f$f.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/$TAG/big_f$f.log
done
echo PHASE_DONE
