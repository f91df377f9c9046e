# Alternating timing runs of several (library / environment / bench args)
# variants on one box (timing only, --cpu-seconds 0):
#   bash tools/ab_multi.sh <tag> <config> <reps> "<name>|<env assignments>|<bench args>" ...
# e.g. "prod||" "occ6|W2V_DEV_LIB=word2vec_amd/lib/occ6/libw2v_hip.so W2V_DEBUG_WPB=8|"
set -o pipefail
TAG=$1; CFG=$2; REPS=$3; shift 3
mkdir -p gpurun_out/$TAG
for r in $(seq $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name envs args <<< "$spec"
    out=gpurun_out/$TAG/${CFG}_${name}_$r
    if ! env $envs timeout -k 10 200 python bench.py --config $CFG --steps 3 --warmup 1 --cpu-seconds 0 $args \
        > $out.json 2> $out.err; then
      echo "$name failed"; tail -3 $out.err; exit 1
    fi
    echo "$CFG $name $r $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
  done
done
