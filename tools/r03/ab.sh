# A/B of two device libraries on the per-pair presets, alternating on one box:
#   bash tools/r03/ab.sh <tag> <variant dir under word2vec_amd/lib> [configs] [reps]
# (the product library is "."; numbers are timing only, with --cpu-seconds 0)
set -o pipefail
TAG=$1; VAR=$2; CONFIGS=${3:-"c3 c2 c1"}; REPS=${4:-2}
mkdir -p gpurun_out/$TAG
run() {  # name lib config
  local lib=$PWD/word2vec_amd/lib/libw2v_hip.so
  [ "$2" != "." ] && lib=$PWD/word2vec_amd/lib/$2/libw2v_hip.so
  W2V_DEV_LIB=$lib timeout -k 10 200 python bench.py --config $3 --steps 3 --warmup 1 --cpu-seconds 0 \
    > gpurun_out/$TAG/$1.json 2> gpurun_out/$TAG/$1.err || { rc=$?; echo "$1 failed rc=$rc"; tail -3 gpurun_out/$TAG/$1.err; return 1; }
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/$TAG/$1.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
}
for r in $(seq $REPS); do
  for c in $CONFIGS; do
    run ${c}_prod_$r . $c || exit 1
    run ${c}_${VAR}_$r $VAR $c || exit 1
  done
done
