# Round 3, lease h: why configs[4] at d512 / neg 15 loses similarity (schedule vs
# formulation vs step size), and the replica split at low saturation thresholds.
set -o pipefail
TAG=${1:-r03h}
mkdir -p gpurun_out/$TAG
# paired-context NS batches: parity (replay / Philox / class, every width) and A/B against one context per batch
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_class.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/$TAG/parity_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
bash tools/r03/ab.sh $TAG nopair "c3" 3 || exit 1
timeout -k 10 500 python -u tools/r03/c5_hot_probe.py -2 11 0,64,2 0 > gpurun_out/$TAG/c5_waves.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_waves.log
timeout -k 10 300 python -u tools/r03/c5_hot_probe.py -2 11 0 0.0125,0.05 > gpurun_out/$TAG/c5_alpha.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_alpha.log
timeout -k 10 900 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8 --rounds 32,128,512 --gmodes split3,split10,split30 > gpurun_out/$TAG/replicas_split.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/replicas_split.log
