# Per-mode throughput under the update policies (default / atomics only /
# plain Hogwild) on one GPU. usage (GPU box): bash tools/mode_policy_sweep.sh
set -o pipefail
mkdir -p gpurun_out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 2 "$@" > gpurun_out/pol_$n.json 2> gpurun_out/pol_$n.err || { tail -5 gpurun_out/pol_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pol_$n.json'));print('$n', round(d['value']/1e6,1), 'M words/s frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'],'ms')"
}
for m in cbow_hs sg_hs cbow_ns; do
  dim=300; [ $m = cbow_hs ] && dim=200
  run ${m}_default --mode $m --dim $dim
  run ${m}_noprivate --mode $m --dim $dim --private-rows 0
  run ${m}_hogwild --mode $m --dim $dim --private-rows 0 --hot-rows 0
done
