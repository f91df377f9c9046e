# Round-end evidence in one lease: smoke(), rocprofv3 kernel-trace +
# FETCH_SIZE + WRITE_SIZE passes of the headline workload, summarised into
# profiles/pmc_traffic.json on the box (copied to gpurun_out/), so that the
# headline bench line that follows (c3, default args: CPU baseline included)
# carries the traffic of this lease and build; then the other presets.
set -o pipefail
TAG=${1:-r02w}
mkdir -p gpurun_out
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || stop smoke $?
bash tools/profile.sh ${TAG}_c3 --config c3 --steps 3 || stop profile $?
python tools/pmc_summary.py ${TAG}_c3 > gpurun_out/${TAG}_pmc_summary.log 2>&1 || stop pmc_summary $?
mkdir -p gpurun_out/${TAG}_profiles && cp profiles/${TAG}_c3_kernel_stats.csv profiles/${TAG}_c3_pmc.json profiles/pmc_traffic.json gpurun_out/${TAG}_profiles/
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || stop bench $?
cat gpurun_out/${TAG}_bench_c3.json
for c in c1 c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || stop bench_$c $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));print('$c',round(d['value']/1e6,2),d['roofline']['frac'],d['roofline']['avg_launch_ms'])"
done
if [ -f word2vec_amd/lib/sn32/libw2v_hip.so ]; then
  W2V_DEV_LIB=$PWD/word2vec_amd/lib/sn32/libw2v_hip.so timeout -k 10 300 python -u bench.py --config c5 --cpu-seconds 0 > gpurun_out/${TAG}_sn32_c5.json 2> gpurun_out/${TAG}_sn32_c5.err && \
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_sn32_c5.json'));print('sn32 c5',round(d['value']/1e6,2),d['roofline']['frac'],d['config']['policy_used'])"
fi
echo PHASE_DONE
