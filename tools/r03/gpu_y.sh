# Round 3, lease y: the whole GPU suite + smoke on the final build (hot-row
# threshold 2), then configs[3]'s per-GPU shard (1.25 B tokens through GPU
# ingestion, one epoch) on it.
set -o pipefail
TAG=${1:-r03y}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/r03/c4_shard.py /tmp/c4_shard.txt > gpurun_out/$TAG/c4_shard.log 2>&1 || { tail -5 gpurun_out/$TAG/c4_shard.log; exit 1; }
cat gpurun_out/$TAG/c4_shard.log
echo PHASE_DONE
