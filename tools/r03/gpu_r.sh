# Round 3, lease r: the whole GPU suite + smoke on the current build, then
# configs[4] LDS-private C rows at negative 15 — throughput (old default 10
# rows vs the new automatic 0) and quality with shorter flush intervals.
set -o pipefail
TAG=${1:-r03r}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
W2V_PARITY_LOG=$PWD/gpurun_out/$TAG/parity_errors.jsonl timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -8; grep -E "shared-negatives c5" gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for pr in 10 -1 10 -1; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --private-rows $pr > gpurun_out/$TAG/c5_pr$pr.json 2> gpurun_out/$TAG/c5_pr$pr.err || exit 1
  echo "c5 private_rows=$pr $(python -c "import json;d=json.load(open('gpurun_out/$TAG/c5_pr$pr.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
done
timeout -k 10 300 python -u tools/r03/c5_hot_probe.py -2 11,12,13 0 0 10 8 256,64 > gpurun_out/$TAG/c5_flush.log 2>&1 || exit 1
cat gpurun_out/$TAG/c5_flush.log
echo PHASE_DONE
