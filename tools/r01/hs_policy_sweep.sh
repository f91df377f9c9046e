# CBOW-HS d200 (configs[1] shape) throughput vs update policy knobs on one GPU.
# usage (GPU box): bash tools/hs_policy_sweep.sh
mkdir -p gpurun_out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --config c2 --cpu-seconds 0 --steps 2 "$@" > gpurun_out/hs_$n.json 2> gpurun_out/hs_$n.err
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$n rc=$rc"; tail -3 gpurun_out/hs_$n.err; exit $rc; fi
  [ $rc -eq 1 ] && { echo "$n: $(tail -1 gpurun_out/hs_$n.err)"; return; }
  python -c "import json;d=json.load(open('gpurun_out/hs_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s', d['roofline']['avg_launch_ms'],'ms')"
}
run default
run ctx_off --context-rows 0
run ctx_flush16 --context-flush 16
run ctx_flush256 --context-flush 256
run ctx_flush1024 --context-flush 1024
run hot0 --hot-rows 0
run cbow_ns_default --mode cbow_ns --dim 200 --negative 5
run cbow_ns_ctx_off --mode cbow_ns --dim 200 --negative 5 --context-rows 0
