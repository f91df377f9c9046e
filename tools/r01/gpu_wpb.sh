# Headline (c3, NV=5) throughput vs workgroup shape at 5 waves/SIMD (experiment knobs).
mkdir -p gpurun_out
run() {  # name, env..., then bench args after --
  local n=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 3 "$@" > gpurun_out/w_$n.json 2> gpurun_out/w_$n.err || { tail -3 gpurun_out/w_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/w_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms frac', d['roofline']['frac'])"
}
run wpb16 X=1 -- --config c3
run wpb4_8k W2V_DEBUG_WPB=4 W2V_DEBUG_LDS_PER_WAVE=8192 -- --config c3
run wpb5_7k W2V_DEBUG_WPB=5 W2V_DEBUG_LDS_PER_WAVE=7168 -- --config c3
run wpb10_7k W2V_DEBUG_WPB=10 W2V_DEBUG_LDS_PER_WAVE=7168 -- --config c3
run wpb4_4k W2V_DEBUG_WPB=4 W2V_DEBUG_LDS_PER_WAVE=4096 -- --config c3
