# Full round evidence on the GPU box: every GPU test, smoke(), one bench line
# per BASELINE config, then rocprofv3 stats + FETCH/WRITE passes per preset.
# usage (GPU box): bash tools/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-r01l}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/bench_configs.sh || exit 1
bash tools/profile_all.sh $TAG || exit 1
