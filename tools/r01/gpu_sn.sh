set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shared.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_shared.log 2>&1 || { tail -30 gpurun_out/gpu_shared.log; exit 1; }
tail -2 gpurun_out/gpu_shared.log
for o in ${SN_OCCS:-0}; do
W2V_SN_OCC=$o timeout -k 10 300 python -u bench.py --mode sg_sn --dim 512 --negative 15 --cpu-seconds 0 --steps 2 > gpurun_out/bench_sn$o.json 2> gpurun_out/bench_sn$o.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_sn$o.json'));print('occ $o', d['value'], d['roofline']['frac'], d['roofline']['mfma']['frac'])"
done
bash tools/sn_prof.sh
