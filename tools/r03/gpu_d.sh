# Round 3, lease d: unguarded whole-row I/O (product) vs the round-2 guards,
# then the parity / class / replica GPU tests on the product library.
set -o pipefail
TAG=${1:-r03d}
mkdir -p gpurun_out/$TAG
bash tools/r03/ab.sh $TAG guards "c3 c2 c1" 2 || { echo "STOP ab"; exit 1; }
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_class.py tests/test_gpu_replicas.py tests/test_gpu_shared.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -12
exit $rc
