# Round-end evidence in one lease (round 3): smoke(), then for every listed
# preset the rocprofv3 kernel-trace + FETCH_SIZE + WRITE_SIZE passes
# (tools/profile.sh), summarised into profiles/pmc_traffic.json on the box (one
# record format for every preset, with its source), then the bench lines, each
# carrying the traffic of this lease and build. The headline (c3, default args)
# runs with the CPU baseline on all host cores.
#   bash tools/r03/final_bench.sh <tag> ["c3 c1 c2 c5"]
set -o pipefail
TAG=${1:-r03z}
PRESETS=${2:-"c3 c1 c2 c5"}
mkdir -p gpurun_out/${TAG}_profiles
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || stop smoke $?
declare -A KEY=([c3]=sg_ns_d300_n50000000 [c1]=sg_ns_d100_n17000000 [c2]=cbow_hs_d200_n17000000 [c5]=sg_sn_d512_n50000000)
for c in $PRESETS; do
  bash tools/profile.sh ${TAG}_$c --config $c --steps 3 || stop profile_$c $?
  python tools/pmc_summary.py ${TAG}_$c ${KEY[$c]} > gpurun_out/${TAG}_pmc_summary_$c.log 2>&1 || stop pmc_summary_$c $?
  cp profiles/${TAG}_${c}_kernel_stats.csv profiles/${TAG}_${c}_pmc.json gpurun_out/${TAG}_profiles/
done
cp profiles/pmc_traffic.json gpurun_out/${TAG}_profiles/
for c in $PRESETS; do
  if [ $c = c3 ]; then
    timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || stop bench $?
  else
    timeout -k 10 300 python -u bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || stop bench_$c $?
  fi
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));print('$c',round(d['value']/1e6,2),d['roofline']['frac'],d['roofline']['avg_launch_ms'],d['roofline']['traffic_source'])"
done
echo PHASE_DONE
