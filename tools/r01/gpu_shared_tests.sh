set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shared.py -x -v --timeout 120 --timeout-method thread -s > gpurun_out/gpu_shared.log 2>&1; rc=$?; tail -30 gpurun_out/gpu_shared.log; exit $rc
