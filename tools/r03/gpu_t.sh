# Round 3, lease t: bounded last-vector row I/O (W2V_ROW_BOUNDED, variant
# library "bounded"): device parity at every row width, then A/B against the
# product on the per-pair presets, alternating.
set -o pipefail
TAG=${1:-r03t}
mkdir -p gpurun_out/$TAG
W2V_DEV_LIB=$PWD/word2vec_amd/lib/bounded/libw2v_hip.so W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/parity_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/$TAG/parity_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
bash tools/r03/ab.sh $TAG bounded "c1 c2 c3" 2 || exit 1
echo PHASE_DONE
