# Round 3, lease i: paired-context SG-NS batches — parity first, then A/B vs one
# context per batch; the saturation-corrected replica exchange (exactness, R = 8 study).
set -o pipefail
TAG=${1:-r03i}
mkdir -p gpurun_out/$TAG
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_class.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/$TAG/parity_tests.log | tail -12
if [ $rc -ne 0 ]; then
  timeout -k 10 120 python -u tools/r03/pair_debug.py gpurun_out/$TAG/pair.npz > gpurun_out/$TAG/pair.log 2>&1 || exit 1
  W2V_DEV_LIB=$PWD/word2vec_amd/lib/nopair/libw2v_hip.so timeout -k 10 120 python -u tools/r03/pair_debug.py gpurun_out/$TAG/nopair.npz > gpurun_out/$TAG/nopair.log 2>&1
  exit 1
fi
bash tools/r03/ab.sh $TAG nopair "c3 c1" 2 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_replicas.py -m gpu -x -v -k "exchange" --timeout 200 --timeout-method thread > gpurun_out/$TAG/replica_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/$TAG/replica_tests.log | tail -6; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/r03/replica_study.py --tokens 50000000 --planted-frac 0.05 --replicas 8 --rounds 64,256 --gmodes sat0.002,sat0.0005 > gpurun_out/$TAG/replicas_sat.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$TAG/replicas_sat.log
echo PHASE_DONE
