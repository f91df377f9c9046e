# Work-item size sweep of the per-pair kernel (W2V_SEG_LEN: tokens of a
# sentence per work item; 0 = whole sentences), then every GPU test at the default.
# usage (GPU box): bash tools/seg_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for c in c1 c2 c3; do
  for L in 0 128 256 512; do
    W2V_SEG_LEN=$L timeout -k 10 200 python -u bench.py --config $c --cpu-seconds 0 > gpurun_out/seg_${c}_$L.json 2> gpurun_out/seg_${c}_$L.err || { tail -5 gpurun_out/seg_${c}_$L.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/seg_${c}_$L.json'));print('$c seg $L', round(d['value']/1e6,2), 'M words/s, kernel ms', d['roofline']['avg_launch_ms'], 'frac', d['roofline']['frac'])"
  done
done | tee gpurun_out/seg_sweep.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
