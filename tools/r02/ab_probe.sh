# A/B of device libraries on one box, alternating, per preset:
#   LIBS="base ." CONFIGS="c3 c2 c1" REPS=2 bash tools/r02/ab_probe.sh <tag>
# ("." is the product library, other names are word2vec_amd/lib/<name>/ variants)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}
mkdir -p gpurun_out/$TAG
for c in ${CONFIGS:-c3 c2 c1}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for v in ${LIBS:-base .}; do
      lib=$R/word2vec_amd/lib/libw2v_hip.so; n=prod
      [ "$v" != "." ] && { lib=$R/word2vec_amd/lib/$v/libw2v_hip.so; n=$v; }
      out=gpurun_out/$TAG/${c}_${n}_$rep
      W2V_DEV_LIB=$lib timeout -k 10 150 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 $BENCH_ARGS \
        > $out.json 2> $out.err || { rc=$?; echo "$c $n failed rc=$rc"; tail -3 $out.err; [ $rc -ge 124 ] && exit 1; continue; }
      echo "$c $n $rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
    done
  done
done
