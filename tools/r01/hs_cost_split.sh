# CBOW-HS (c2): where the update policy's time goes (throughput only).
# usage (GPU box): bash tools/hs_cost_split.sh
set -o pipefail
mkdir -p gpurun_out
run() {
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --config c2 --cpu-seconds 0 "$@" > gpurun_out/hc_$n.json 2> gpurun_out/hc_$n.err || { tail -5 gpurun_out/hc_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/hc_$n.json'));print('c2 $n', round(d['value']/1e6,2), 'M words/s')"
}
{
run default
run hot0 --hot-rows 0
run priv_off --private-rows 0
run ctx_off --context-rows 0
run priv_ctx_off --private-rows 0 --context-rows 0
run plain --hot-rows 0 --private-rows 0 --context-rows 0
run flush128 --flush-centers 128
run ctxflush64 --context-flush 64
} | tee gpurun_out/hs_cost_split.log
