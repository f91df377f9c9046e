# Timing-only bound: what the memory-side atomics cost the per-pair kernel.
# Variants from tools/r02/exp_variant.sh skip<k> "-DW2V_EXP_SKIP=<k>" (numerics
# wrong by construction): 1 = no hot-row target atomics, 2 = no private-row
# flush atomics, 4 = no hot context-row atomics (CBOW), 7 = none of them.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/skip
run() {  # tag lib config
  local lib=$R/word2vec_amd/lib/libw2v_hip.so
  [ "$2" != "." ] && lib=$R/word2vec_amd/lib/$2/libw2v_hip.so
  W2V_DEV_LIB=$lib timeout -k 10 150 python bench.py --config $3 --steps 3 --warmup 1 --cpu-seconds 0 \
    > gpurun_out/skip/$1.json 2> gpurun_out/skip/$1.err || { rc=$?; echo "$1 failed rc=$rc"; tail -3 gpurun_out/skip/$1.err; [ $rc -ge 124 ] && return 1; return 0; }
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/skip/$1.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
}
for c in ${CONFIGS:-c2 c3}; do
  for v in . skip1 skip2 skip4 skip7; do
    [ "$c" = c3 ] && [ "$v" = skip4 ] && continue
    run ${c}_${v#.} $v $c || exit 1
  done
done
