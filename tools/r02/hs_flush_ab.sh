# configs[1] (CBOW-HS): automatic flush interval (default) against the fixed
# round-1 intervals (nodes 64 / context rows 32), alternating on one box.
#   REPS=2 bash tools/r02/hs_flush_ab.sh <tag>
set -o pipefail
TAG=${1:-hsab}
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 ${REPS:-2}); do
  for v in auto fixed; do
    extra=""; [ $v = fixed ] && extra="--flush-centers 64 --context-flush 32"
    out=gpurun_out/$TAG/c2_${v}_$rep
    timeout -k 10 150 python bench.py --config c2 --steps 3 --warmup 1 --cpu-seconds 0 $extra > $out.json 2> $out.err \
      || { rc=$?; echo "c2 $v failed rc=$rc"; tail -3 $out.err; exit 1; }
    echo "c2 $v $rep $(python -c "import json;d=json.load(open('$out.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'],d['config']['policy_used'])")"
  done
done
