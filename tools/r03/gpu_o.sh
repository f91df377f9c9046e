# Round 3, lease o: the whole GPU suite once (nothing deselected) and smoke().
set -o pipefail
TAG=${1:-r03o}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -12; grep -E "^replicas " gpurun_out/$TAG/gpu_tests.log
exit $rc
