# Round 3, lease x: the large-vocabulary hot-row threshold 2 (was 4): quality at
# the headline's scale through the automatic rule (3 seeds), the headline
# profile (kernel-trace + FETCH/WRITE) and bench line on this build.
set -o pipefail
TAG=${1:-r03x}
mkdir -p gpurun_out/$TAG gpurun_out/${TAG}_profiles
timeout -k 10 300 python -u tools/r03/replica_study.py --tokens 50000000 --filler 1000000 --dim 300 --planted-frac 0.05 --replicas "" --seeds 1,2,3 > gpurun_out/$TAG/quality_auto.log 2>&1 || exit 1
grep '"R": 1' gpurun_out/$TAG/quality_auto.log
bash tools/profile.sh ${TAG}_c3 --config c3 --steps 3 || exit 1
python tools/pmc_summary.py ${TAG}_c3 sg_ns_d300_n50000000 > gpurun_out/$TAG/pmc_summary_c3.log 2>&1 || exit 1
cp profiles/${TAG}_c3_kernel_stats.csv profiles/${TAG}_c3_pmc.json profiles/pmc_traffic.json gpurun_out/${TAG}_profiles/
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.err || exit 1
cat gpurun_out/$TAG/bench_c3.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_quality.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/quality_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/quality_tests.log; [ $rc -eq 0 ] || exit 1
echo PHASE_DONE
