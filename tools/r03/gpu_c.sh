# Round 3, lease c: the changed GPU tests (replicas incl. the adaptive exchange and
# the one-rank RCCL path, parity, class checkpoints, quality gates), the
# 8-replica exchange study on two corpus difficulties, and the configs[3]
# per-GPU shard (1.25 B tokens through GPU ingestion).
set -o pipefail
TAG=${1:-r03c}
mkdir -p gpurun_out/$TAG
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 900 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_parity.py tests/test_gpu_class.py tests/test_gpu_quality.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|^paired|^planted|^replicas|^shared" gpurun_out/$TAG/gpu_tests.log | tail -40
[ $rc -le 1 ] || stop gpu_tests $rc
for f in 0.01 0.03; do
  timeout -k 10 600 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac $f --replicas 8 --rounds 1,4,16,64 --gmodes adaptive,average,sum > gpurun_out/$TAG/replicas_f$f.log 2>&1 || stop replicas $?
  grep -v amdgpu.ids gpurun_out/$TAG/replicas_f$f.log
done
df -h /tmp . | tail -2
timeout -k 10 900 python -u tools/r03/c4_shard.py /tmp/w2v_c4_shard.txt > gpurun_out/$TAG/c4_shard.log 2>&1; rc=$?
rm -f /tmp/w2v_c4_shard.txt
cat gpurun_out/$TAG/c4_shard.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || stop c4_shard $rc
