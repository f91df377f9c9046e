# A/B of two bench.py argument sets on one box, alternating (timing only, --cpu-seconds 0):
#   bash tools/ab_args.sh <tag> <config> "<args A>" "<args B>" [reps]
set -o pipefail
TAG=$1; CFG=$2; A=$3; B=$4; REPS=${5:-3}
mkdir -p gpurun_out/$TAG
run() {  # name args
  timeout -k 10 200 python bench.py --config $CFG --steps 3 --warmup 1 --cpu-seconds 0 $2 \
    > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || { rc=$?; echo "$1 failed rc=$rc"; tail -3 gpurun_out/$TAG/$1.err; return 1; }
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/$TAG/$1.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
}
for r in $(seq $REPS); do
  run ${CFG}_A_$r "$A" || exit 1
  run ${CFG}_B_$r "$B" || exit 1
done
