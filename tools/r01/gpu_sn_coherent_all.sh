# Shared-negatives: quality (text8-like, 3 seeds) and speed vs the rows that
# take atomic deltas (hot_rows; W2V_SN_ATOMIC_ROWS overrides for experiments).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shared.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sn_tests.log 2>&1 || { tail -20 gpurun_out/sn_tests.log; exit 1; }
tail -1 gpurun_out/sn_tests.log
timeout -k 10 400 python -u tools/sn_zipf_concurrency.py 0 32 > gpurun_out/snhot.log 2>&1 || { cat gpurun_out/snhot.log; exit 1; }
cat gpurun_out/snhot.log
for h in 1000 0 100 10000; do W2V_SN_ATOMIC_ROWS=$h timeout -k 10 200 python -u bench.py --config c5 --cpu-seconds 0 --steps 2 > gpurun_out/c5_h$h.json 2>gpurun_out/c5_h$h.err || exit 1; python -c "import json;d=json.load(open('gpurun_out/c5_h$h.json'));print('atomic rows $h', round(d['value']/1e6,1))"; done
