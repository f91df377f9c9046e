set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/sn_zipf_concurrency.py > gpurun_out/sn_zipf_conc.log 2>&1 || { tail -20 gpurun_out/sn_zipf_conc.log; exit 1; }
cat gpurun_out/sn_zipf_conc.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 2 "$@" > gpurun_out/c3_$n.json 2> gpurun_out/c3_$n.err || { tail -3 gpurun_out/c3_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c3_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms')"
}
run default
run hot64 --hot-rows 64
run hot0 --hot-rows 0
run hogwild --hot-rows 0 --private-rows 0
run c2 --config c2
