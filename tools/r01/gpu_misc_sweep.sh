# Speed sweeps: c1 (SG-NS d100) policy cost; c5 coherent-row count.
mkdir -p gpurun_out
run() {  # name, env, args...
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 2 "$@" > gpurun_out/m_$n.json 2> gpurun_out/m_$n.err || { tail -3 gpurun_out/m_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/m_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms frac', d['roofline']['frac'])"
}
run c1 X=1 --config c1
run c1_hot0 X=1 --config c1 --hot-rows 0
run c1_hogwild X=1 --config c1 --hot-rows 0 --private-rows 0
run c1_V1M X=1 --config c1 --vocab 1000000 --tokens 50000000
run c5_coh1000 W2V_SN_COHERENT_ROWS=1000 --config c5
run c5_coh16384 W2V_SN_COHERENT_ROWS=16384 --config c5
run c5 X=1 --config c5
