# A/B of the dedicated flush wave (W2V_FLUSH_WAVE=1) against the in-line
# flush on the same library, alternating, per preset:
#   LIB=fw CONFIGS="c2 c3" REPS=2 bash tools/r02/flush_wave_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-fwab}
lib=$R/word2vec_amd/lib/${LIB:-fw}/libw2v_hip.so
mkdir -p gpurun_out/$TAG
for c in ${CONFIGS:-c2 c3}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for fw in 0 1; do
      out=gpurun_out/$TAG/${c}_fw${fw}_$rep
      W2V_FLUSH_WAVE=$fw W2V_DEV_LIB=$lib timeout -k 10 150 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 \
        > $out.json 2> $out.err || { rc=$?; echo "$c fw$fw failed rc=$rc"; tail -3 $out.err; exit 1; }
      echo "$c fw$fw $rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['env_knobs'])")"
    done
  done
done
