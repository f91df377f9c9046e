# Every GPU test, then one bench line per BASELINE config preset.
# usage (GPU box): bash tools/gpu_tests_bench.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
grep -E "^(planted|text8)" -h gpurun_out/gpu_tests.log || true
CPU_SECONDS=${CPU_SECONDS:-6} bash tools/bench_configs.sh
