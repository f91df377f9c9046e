# Headline (c3) speed vs private-row flush interval and atomic rows.
mkdir -p gpurun_out
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --config c3 --cpu-seconds 0 --steps 3 "$@" > gpurun_out/nf_$n.json 2> gpurun_out/nf_$n.err || { tail -2 gpurun_out/nf_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/nf_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms')"
}
run default
run flush64 --flush-centers 64
run flush1024 --flush-centers 1024
run flush4096 --flush-centers 4096
run private0 --private-rows 0
run hot0 --hot-rows 0
