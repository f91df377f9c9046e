# One short bench line per preset (default c3 c2 c1) with the product library:
#   CONFIGS="c3 c2" bash tools/r02/bench_quick.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-quick}; shift
mkdir -p gpurun_out/$TAG
for c in ${CONFIGS:-c3 c2 c1}; do
  timeout -k 10 150 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 "$@" \
    > gpurun_out/$TAG/$c.json 2> gpurun_out/$TAG/$c.err || { rc=$?; echo "$c failed rc=$rc"; tail -3 gpurun_out/$TAG/$c.err; exit 1; }
  echo "$c $(python -c "import json;d=json.load(open('gpurun_out/$TAG/$c.json'));print(round(d['value']/1e6,2),d['roofline']['frac'],d['ms_per_step'])")"
done
