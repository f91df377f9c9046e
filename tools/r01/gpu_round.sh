# Round GPU check: every GPU test, then the headline bench (configs[2]) and the
# configs[4] shared-negatives bench. usage (GPU box): bash tools/gpu_round.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
timeout -k 10 300 python -u bench.py --mode sg_sn --dim 512 --negative 15 --cpu-seconds 5 > gpurun_out/bench_sn.json 2> gpurun_out/bench_sn.err || exit 1
cat gpurun_out/bench_sn.json
