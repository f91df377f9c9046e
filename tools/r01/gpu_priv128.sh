# Up to 128 LDS-private output rows: parity + quality gates, then preset speeds and private-row counts.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_quality.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/p128.log 2>&1 || { grep -E "planted|text8|passed|failed|Error" gpurun_out/p128.log | tail -12; exit 1; }
grep -E "planted|text8|passed|failed" gpurun_out/p128.log | tail -12
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 3 "$@" > gpurun_out/p_$n.json 2> gpurun_out/p_$n.err || { tail -2 gpurun_out/p_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/p_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms')"
}
run c3 --config c3
run c3_p128 --config c3 --private-rows 128
run c1 --config c1
run c1_p128 --config c1 --private-rows 128
run c2 --config c2
