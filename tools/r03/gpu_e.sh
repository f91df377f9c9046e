# Round 3, lease e: A/B (atomics masked, loads/stores whole rows) vs the round-2
# guards; the replica-exchange study with the frequency split.
set -o pipefail
TAG=${1:-r03e}
mkdir -p gpurun_out/$TAG
bash tools/r03/ab.sh $TAG guards "c3 c2 c1" 2 || { echo "STOP ab"; exit 1; }
for f in 0.05; do
  timeout -k 10 800 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac $f --replicas 8 --rounds 8,32,128 --gmodes split100,split1000,split10000,adaptive,average > gpurun_out/$TAG/replicas_f$f.log 2>&1 || { echo "STOP replicas"; exit 1; }
  grep -v amdgpu.ids gpurun_out/$TAG/replicas_f$f.log
done
timeout -k 10 300 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 2 --rounds 64 --gmodes sum,split1000 > gpurun_out/$TAG/replicas_r2.log 2>&1 || { echo "STOP r2"; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/replicas_r2.log
