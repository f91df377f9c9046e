# Round-end evidence, part A (round 3): smoke(), the whole GPU suite once
# (nothing deselected), then the headline (c3): rocprofv3 kernel-trace +
# FETCH_SIZE + WRITE_SIZE passes summarised into profiles/pmc_traffic.json on
# the box, and the bench line carrying that traffic (CPU baseline on all cores).
set -o pipefail
TAG=${1:-r03z}
mkdir -p gpurun_out/${TAG}_profiles
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/${TAG}_smoke.log
W2V_PARITY_LOG=$PWD/gpurun_out/${TAG}_parity_errors.jsonl timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_gpu_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || stop gpu_tests $rc
bash tools/profile.sh ${TAG}_c3 --config c3 --steps 3 || stop profile_c3 $?
python tools/pmc_summary.py ${TAG}_c3 sg_ns_d300_n50000000 > gpurun_out/${TAG}_pmc_summary_c3.log 2>&1 || stop pmc_summary_c3 $?
cp profiles/${TAG}_c3_kernel_stats.csv profiles/${TAG}_c3_pmc.json profiles/pmc_traffic.json gpurun_out/${TAG}_profiles/
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || stop bench $?
cat gpurun_out/${TAG}_bench_c3.json
echo PHASE_DONE
