set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shared.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_shared.log 2>&1 || { tail -30 gpurun_out/gpu_shared.log; exit 1; }
tail -3 gpurun_out/gpu_shared.log
timeout -k 10 300 python -u bench.py --mode sg_sn --dim 512 --negative 15 --cpu-seconds 5 > gpurun_out/bench_sn.json 2> gpurun_out/bench_sn.err && cat gpurun_out/bench_sn.json
