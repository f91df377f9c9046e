# Round 3, last lease: the configs[4] own-hyper-parameter gate (5 seeds) and
# configs[3]'s per-GPU shard (1.25 B tokens through GPU ingestion, one epoch)
# on the final build.
set -o pipefail
TAG=${1:-r03z2}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_quality.py -m gpu -v -s -k c5_hyperparameters --timeout 280 --timeout-method thread > gpurun_out/$TAG/c5_gate.log 2>&1
rc=$?; grep -E "shared-negatives c5|passed|failed" gpurun_out/$TAG/c5_gate.log | tail -3; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/r03/c4_shard.py /tmp/c4_shard.txt > gpurun_out/$TAG/c4_shard.log 2>&1 || { tail -5 gpurun_out/$TAG/c4_shard.log; exit 1; }
cat gpurun_out/$TAG/c4_shard.log
echo PHASE_DONE
