# Round-end evidence, part B (round 3): configs[0], [1], [4] — rocprofv3
# kernel-trace + FETCH_SIZE + WRITE_SIZE passes, then their bench lines with
# this lease's traffic; configs[4] with the old 10 LDS-private rows beside the
# new automatic setting (none above negative 5), alternating.
set -o pipefail
TAG=${1:-r03z}
mkdir -p gpurun_out/${TAG}_profiles
stop() { echo "STOP after $1 (rc=$2)"; exit 1; }
declare -A KEY=([c1]=sg_ns_d100_n17000000 [c2]=cbow_hs_d200_n17000000 [c5]=sg_sn_d512_n50000000)
for c in c1 c2 c5; do
  bash tools/profile.sh ${TAG}_$c --config $c --steps 3 || stop profile_$c $?
  python tools/pmc_summary.py ${TAG}_$c ${KEY[$c]} > gpurun_out/${TAG}_pmc_summary_$c.log 2>&1 || stop pmc_summary_$c $?
  cp profiles/${TAG}_${c}_kernel_stats.csv profiles/${TAG}_${c}_pmc.json gpurun_out/${TAG}_profiles/
done
cp profiles/pmc_traffic.json gpurun_out/${TAG}_profiles/
for c in c1 c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || stop bench_$c $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$c.json'));print('$c',round(d['value']/1e6,2),d['roofline']['frac'],d['roofline']['avg_launch_ms'],d['roofline']['traffic_source'])"
done
for pr in 10 -1 10 -1; do
  timeout -k 10 200 python bench.py --config c5 --steps 3 --warmup 1 --cpu-seconds 0 --private-rows $pr > gpurun_out/${TAG}_c5_pr$pr.json 2> gpurun_out/${TAG}_c5_pr$pr.err || stop c5_pr $?
  echo "c5 private_rows=$pr $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_c5_pr$pr.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
done
# the headline line again with the CPU baseline on the usable cores (affinity capped by the cgroup quota)
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || stop bench_c3 $?
cat gpurun_out/${TAG}_bench_c3.json
echo PHASE_DONE
