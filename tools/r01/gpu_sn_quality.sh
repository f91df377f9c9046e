# configs[4] shared-negatives: parity tests, bench, and quality against the
# per-pair oracle goldens (tools/quality_shared.py). usage (GPU box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shared.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_shared.log 2>&1 || { tail -30 gpurun_out/gpu_shared.log; exit 1; }
tail -1 gpurun_out/gpu_shared.log
timeout -k 10 200 python -u bench.py --mode sg_sn --dim 512 --negative 15 --cpu-seconds 0 --steps 2 > gpurun_out/bench_sn.json 2> gpurun_out/bench_sn.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_sn.json'));print('sn', d['value'], d['roofline']['frac'], d['roofline']['mfma']['frac'])"
timeout -k 10 500 python -u tools/quality_shared.py > gpurun_out/qshared.log 2>&1; grep shared=True gpurun_out/qshared.log
